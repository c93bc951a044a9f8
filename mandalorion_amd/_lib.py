"""ctypes binding of libmando.so (the C-ABI declared in include/mando.h).

The product path is HIP-only: if the shared library is missing, or no gfx950 device is visible,
every compute entry point raises instead of falling back to a CPU implementation.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libmando.so")

# Every symbol include/mando.h declares (tests check the library exports all of them).
EXPORTED = (
    "mando_last_error",
    "mando_abi_version",
    "mando_poa_default_params",
    "mando_device_count",
    "mando_ctx_create",
    "mando_ctx_destroy",
    "mando_ctx_blocking_sync",
    "mando_poa_batch",
    "mando_poa_batch_device",
    "mando_ctx_sync",
    "mando_last_kernel_ms",
    "mando_last_kernel_launches",
    "mando_ctx_set_poa_budget",
    "mando_ctx_memory",
    "mando_device_memory",
    "mando_cache_trim",
    "mando_poa_last_slots",
    "mando_orient_batch",
    "mando_selftest",
    "mando_mt_permutation",
    "mando_cluster_default_params",
    "mando_cluster_loci",
    "mando_cluster_view_get",
    "mando_cluster_free",
    "mando_cluster_device_text",
    "mando_orient_segments",
    "mando_poa_segments",
    "mando_comm_init",
    "mando_comm_backend",
    "mando_allgather_counts",
    "mando_allgather_bytes",
    "mando_gather_bytes",
    "mando_allreduce_max_f64",
    "mando_comm_barrier",
    "mando_comm_destroy",
    "mando_rccl_allgather_plan",
    "mando_rccl_gather_plan",
    "mando_rccl_alltoallv_plan",
    "mando_alltoallv_bytes",
    "mando_pack_segments",
    "mando_format_outputs",
    "mando_write_blocks",
    "mando_split_loci",
    "mando_split_loci_device",
    "mando_list_roots",
    "mando_list_root_names",
    "mando_root_sizes",
    "mando_sam_to_psl",
    "mando_sam_to_psl_device",
    "mando_clean_psl",
    "mando_filter_default_params",
    "mando_filter_sam",
    "mando_filter_isoforms",
    "mando_filter_isoforms_device",
    "mando_psl_to_gtf",
    "mando_quantify",
    "mando_quantify_device",
)

STATUS = {
    0: "MANDO_OK",
    -1: "MANDO_E_ARG",
    -2: "MANDO_E_HIP",
    -3: "MANDO_E_NOMEM",
    -4: "MANDO_E_CAP",
    -5: "MANDO_E_UNSUPPORTED",
    -6: "MANDO_E_INTERNAL",
    -7: "MANDO_E_NODEV",
}


class MandoError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


class PoaParams(ctypes.Structure):
    """mando_poa_params — defaults are the reference's `abpoa -M 5 -r 0`."""

    _fields_ = [
        ("match", ctypes.c_int32),
        ("mismatch", ctypes.c_int32),
        ("gap_open1", ctypes.c_int32),
        ("gap_ext1", ctypes.c_int32),
        ("gap_open2", ctypes.c_int32),
        ("gap_ext2", ctypes.c_int32),
        ("band_b", ctypes.c_int32),
        ("band_f", ctypes.c_float),
        ("seeding", ctypes.c_int32),
        ("k", ctypes.c_int32),
        ("w", ctypes.c_int32),
        ("min_w", ctypes.c_int32),
    ]

    @classmethod
    def defaults(cls) -> "PoaParams":
        p = cls()
        load().mando_poa_default_params(ctypes.byref(p))
        return p


class ClusterParams(ctypes.Structure):
    """mando_cluster_params — defaults are Mando.py's D-module arguments (Mando.py:382-399)."""

    _fields_ = [
        ("cutoff", ctypes.c_double),
        ("splice_site_width", ctypes.c_int32),
        ("minimum_read_count", ctypes.c_int32),
        ("upstream_buffer", ctypes.c_int32),
        ("downstream_buffer", ctypes.c_int32),
        ("junctions", ctypes.c_char_p),
        ("seed", ctypes.c_uint32),
        ("threads", ctypes.c_int32),
        ("poa_subsample", ctypes.c_int32),
        ("orient_ctx", ctypes.c_void_p),
        ("orient_max_hits", ctypes.c_int32),
    ]

    @classmethod
    def defaults(cls) -> "ClusterParams":
        p = cls()
        load().mando_cluster_default_params(ctypes.byref(p))
        return p


class ClusterView(ctypes.Structure):
    _fields_ = [
        ("n_loci", ctypes.c_int64),
        ("locus_status", ctypes.POINTER(ctypes.c_int32)),
        ("text", ctypes.c_void_p),
        ("text_len", ctypes.c_int64),
        ("n_records", ctypes.c_int64),
        ("name_off", ctypes.POINTER(ctypes.c_int64)),
        ("name_len", ctypes.POINTER(ctypes.c_int32)),
        ("seq_off", ctypes.POINTER(ctypes.c_int64)),
        ("seq_len", ctypes.POINTER(ctypes.c_int32)),
        ("rec_locus", ctypes.POINTER(ctypes.c_int64)),
        ("n_isoforms", ctypes.c_int64),
        ("iso_locus", ctypes.POINTER(ctypes.c_int64)),
        ("mem_off", ctypes.POINTER(ctypes.c_int64)),
        ("mem", ctypes.POINTER(ctypes.c_int64)),
        ("sub_off", ctypes.POINTER(ctypes.c_int64)),
        ("sub", ctypes.POINTER(ctypes.c_int64)),
        ("n_peaks", ctypes.c_int64),
        ("peak_locus", ctypes.POINTER(ctypes.c_int64)),
        ("peak_start", ctypes.POINTER(ctypes.c_int64)),
        ("peak_end", ctypes.POINTER(ctypes.c_int64)),
        ("peak_type", ctypes.POINTER(ctypes.c_char)),
        ("peak_side", ctypes.POINTER(ctypes.c_char)),
        ("peak_prop", ctypes.POINTER(ctypes.c_double)),
        ("orient_max_hits", ctypes.c_int32),
        ("orient_hits", ctypes.POINTER(ctypes.c_int8)),
        ("orient_n_hits", ctypes.POINTER(ctypes.c_int32)),
    ]


_lib = None
_lock = threading.Lock()
_P = ctypes.c_void_p
_I64 = ctypes.c_int64


def load(path: str | None = None):
    """Load libmando.so and declare argument types.  Raises if the library is absent."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or os.environ.get("MANDO_LIB") or LIB_PATH
        if not os.path.exists(p):
            raise MandoError(-7, f"{p} not built (run __graft_entry__.build() or make -C mandalorion_amd/csrc)")
        lib = ctypes.CDLL(p)
        lib.mando_last_error.restype = ctypes.c_char_p
        lib.mando_last_error.argtypes = []
        lib.mando_abi_version.restype = ctypes.c_int
        lib.mando_poa_default_params.argtypes = [_P]
        lib.mando_poa_default_params.restype = None
        lib.mando_device_count.argtypes = [_P]
        lib.mando_ctx_create.argtypes = [ctypes.c_int, _P]
        lib.mando_ctx_destroy.argtypes = [_P]
        lib.mando_ctx_destroy.restype = None
        lib.mando_ctx_sync.argtypes = [_P]
        lib.mando_poa_batch.argtypes = [_P, _P, _P, _P, _P, _I64, _P, _P, _I64, _P, _P]
        lib.mando_poa_batch_device.argtypes = [_P, _P, _P, _P, _P, _I64, _I64, _I64, _P, _P, _P, _P, _P]
        lib.mando_last_kernel_ms.argtypes = [_P]
        lib.mando_last_kernel_ms.restype = ctypes.c_float
        lib.mando_last_kernel_launches.argtypes = [_P]
        lib.mando_ctx_set_poa_budget.argtypes = [_P, _I64]
        lib.mando_ctx_memory.argtypes = [_P, _P, _P]
        lib.mando_device_memory.argtypes = [ctypes.c_int, _P, _P]
        lib.mando_cache_trim.argtypes = [ctypes.c_int, _I64, _I64, _P]
        lib.mando_poa_last_slots.argtypes = [_P, _P, _P]
        lib.mando_orient_batch.argtypes = [_P, _P, _P, _P, _I64, _P, ctypes.c_int32, _P]
        lib.mando_mt_permutation.argtypes = [ctypes.c_uint32, _P, _P, _I64, _P, _I64]
        lib.mando_cluster_default_params.argtypes = [_P]
        lib.mando_cluster_default_params.restype = None
        lib.mando_cluster_loci.argtypes = [_P, _P, _P, _P, _I64, _P, _P, _P]
        lib.mando_cluster_view_get.argtypes = [_P, _P]
        lib.mando_cluster_free.argtypes = [_P]
        lib.mando_cluster_free.restype = None
        lib.mando_cluster_device_text.argtypes = [_P, _P, _P]
        lib.mando_orient_segments.argtypes = [_P, _P, _I64, _P, _P, _P, _I64, _P, ctypes.c_int32, _P]
        lib.mando_poa_segments.argtypes = [_P, _P, _P, _I64, _P, _P, _P, _P, _I64, _P, _P, _I64, _P, _P]
        lib.mando_split_loci.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int32, ctypes.c_char_p, _P, _P]
        lib.mando_split_loci_device.argtypes = [_P, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int32, ctypes.c_char_p,
                                                _P, _P]
        lib.mando_list_roots.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, _P,
                                         ctypes.c_int64, _P, _P]
        lib.mando_list_root_names.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int64, _P, _P]
        lib.mando_root_sizes.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, _P]
        lib.mando_sam_to_psl.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, _P]
        lib.mando_sam_to_psl_device.argtypes = [_P, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int32, _P]
        lib.mando_clean_psl.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int32, _P]
        lib.mando_filter_default_params.argtypes = [_P]
        lib.mando_filter_default_params.restype = None
        lib.mando_filter_sam.argtypes = [ctypes.c_char_p, ctypes.c_char_p, _P]
        lib.mando_filter_isoforms.argtypes = [_P] + [ctypes.c_char_p] * 7 + [_P]
        lib.mando_filter_isoforms_device.argtypes = [_P, _P] + [ctypes.c_char_p] * 7 + [_P]
        lib.mando_psl_to_gtf.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        lib.mando_quantify.argtypes = [_P, ctypes.c_int32] + [ctypes.c_char_p] * 4
        lib.mando_quantify_device.argtypes = [_P, _P, ctypes.c_int32] + [ctypes.c_char_p] * 4
        lib.mando_pack_segments.argtypes = [_P, _P, _P, _P, _P, _I64, _P, _P, ctypes.c_int32]
        lib.mando_format_outputs.argtypes = [_I64, _I64] + [_P] * 12 + [_P, _I64, _P, _P, _I64, _P, _P, _P,
                                                                         ctypes.c_int32]
        lib.mando_write_blocks.argtypes = [ctypes.c_int32, _P, _P, _P, _P, _I64, ctypes.c_int32]
        lib.mando_comm_init.argtypes = [_P, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                        ctypes.c_double, _P]
        lib.mando_comm_backend.argtypes = [_P]
        lib.mando_allgather_counts.argtypes = [_P, _I64, _P]
        lib.mando_allgather_bytes.argtypes = [_P, _P, _I64, _P, _P]
        lib.mando_gather_bytes.argtypes = [_P, _P, _I64, _P, _P]
        lib.mando_allreduce_max_f64.argtypes = [_P, _P]
        lib.mando_comm_barrier.argtypes = [_P]
        lib.mando_comm_destroy.argtypes = [_P]
        lib.mando_comm_destroy.restype = None
        if hasattr(lib, "mando_rccl_gather_plan"):  # (dev A/B builds of older trees lack them)
            lib.mando_rccl_allgather_plan.argtypes = [ctypes.c_int, _P, _P, _P, _P]
            lib.mando_rccl_gather_plan.argtypes = [ctypes.c_int, ctypes.c_int, _P, _P, _P, _P, _P]
        if hasattr(lib, "mando_alltoallv_bytes"):
            lib.mando_rccl_alltoallv_plan.argtypes = [ctypes.c_int, _P, _P, _P, _P]
            lib.mando_alltoallv_bytes.argtypes = [_P, _P, _P, _P, _P]
        if hasattr(lib, "mando_selftest"):
            lib.mando_selftest.argtypes = [_P, _P]
        if path is None:
            _lib = lib
        return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = load().mando_last_error()
        raise MandoError(rc, msg.decode() if msg else "")


def device_count() -> int:
    n = ctypes.c_int(0)
    check(load().mando_device_count(ctypes.byref(n)))
    return n.value


def ptr(a: np.ndarray | None) -> int | None:
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def pack_segments(srcs: list[np.ndarray], starts: np.ndarray, lens: np.ndarray, sel: np.ndarray | None = None,
                  rc: np.ndarray | None = None, threads: int = 0, out: np.ndarray | None = None,
                  out_off: np.ndarray | None = None) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate byte segments of the uint8 arrays in srcs (see mando_pack_segments); returns
    (bytes uint8 array, offsets int64 with n+1 entries).  With out / out_off: segment i goes to
    out[out_off[i]:] instead (a scatter; out is returned as is)."""
    lib = load()
    n = int(len(starts))
    lens = np.ascontiguousarray(lens, dtype=np.int64)
    if out is not None:
        off = np.ascontiguousarray(out_off, dtype=np.int64)
        if len(off) != n or (n and int((off + lens).max()) > out.size) or (n and int(off.min()) < 0):
            raise ValueError("pack_segments: a segment falls outside out")
    else:
        off = np.zeros(n + 1, dtype=np.int64)
        if n:
            np.cumsum(lens, out=off[1:])
        out = np.empty(max(int(off[-1]), 1), dtype=np.uint8)
    if n == 0:
        return (out if out_off is not None else out[:0]), off
    if len(srcs) > 127:
        raise ValueError("pack_segments: at most 127 sources (int8 selectors)")
    keep = [np.ascontiguousarray(s, dtype=np.uint8) for s in srcs]
    ptrs = (ctypes.c_void_p * len(keep))(*[k.ctypes.data for k in keep])
    starts = np.ascontiguousarray(starts, dtype=np.int64)
    sel_a = None if sel is None else np.ascontiguousarray(sel, dtype=np.int8)
    rc_a = None if rc is None else np.ascontiguousarray(rc, dtype=np.int8)
    check(lib.mando_pack_segments(ptrs, ptr(sel_a), ptr(starts), ptr(lens), ptr(rc_a), n, ptr(out), ptr(off), threads))
    if out_off is not None:
        return out, off
    return out[:int(off[-1])], off


def format_outputs(order: np.ndarray, mem_off: np.ndarray, counter0: int, cons: tuple | None, names: tuple | None,
                   threads: int = 0, iso_k: np.ndarray | None = None, offsets: bool = False):
    """The Isoform_Consensi.fasta and reads2isoforms.txt bytes of the isoforms `order` (see
    mando_format_outputs).  cons = (srcs, sel, start, len, rc), names = (srcs, sel, start, len); either None
    skips that file.  iso_k: each output isoform's number (default counter0 + 1 + position).  Returns
    (fasta bytes or None, r2i bytes or None) as uint8 arrays, plus both files' per-isoform start offsets
    (n + 1 entries each) when offsets."""
    lib = load()
    order = np.ascontiguousarray(order, dtype=np.int64)
    mem_off = np.ascontiguousarray(mem_off, dtype=np.int64)
    kk = None if iso_k is None else np.ascontiguousarray(iso_k, dtype=np.int64)
    if kk is not None and len(kk) != len(order):
        raise ValueError("format_outputs: iso_k and order differ in length")
    keep = []

    def srcs_of(lst):
        k = [np.ascontiguousarray(s, dtype=np.uint8) for s in lst]
        keep.extend(k)
        return (ctypes.c_void_p * max(len(k), 1))(*[x.ctypes.data for x in k])

    def arr(a, dt):
        return None if a is None else np.ascontiguousarray(a, dtype=dt)

    c = [None] * 5 if cons is None else [srcs_of(cons[0]), arr(cons[1], np.int16), arr(cons[2], np.int64),
                                          arr(cons[3], np.int64), arr(cons[4], np.int8)]
    n = [None] * 4 if names is None else [srcs_of(names[0]), arr(names[1], np.int16), arr(names[2], np.int64),
                                           arr(names[3], np.int64)]
    fl, rl = ctypes.c_int64(0), ctypes.c_int64(0)
    fo = np.empty(len(order) + 1, np.int64)
    ro = np.empty(len(order) + 1, np.int64)

    def call(fa, fcap, r2, rcap):
        return lib.mando_format_outputs(len(order), counter0, ptr(kk), ptr(order), ptr(mem_off), c[0], ptr(c[1]),
                                        ptr(c[2]), ptr(c[3]), ptr(c[4]), n[0], ptr(n[1]), ptr(n[2]), ptr(n[3]),
                                        fa, fcap, ctypes.byref(fl), r2, rcap, ctypes.byref(rl), ptr(fo), ptr(ro),
                                        threads)

    # sizes first (zero capacities: MANDO_E_CAP with both lengths set), then the fill
    dummy = ctypes.c_uint8()
    rc = call(ctypes.byref(dummy) if cons is not None else None, 0,
              ctypes.byref(dummy) if names is not None else None, 0)
    if rc not in (0, -4):
        check(rc)
    fasta = np.empty(max(fl.value, 1), np.uint8) if cons is not None else None
    r2i = np.empty(max(rl.value, 1), np.uint8) if names is not None else None
    check(call(ptr(fasta), fl.value if fasta is not None else 0, ptr(r2i), rl.value if r2i is not None else 0))
    out = (None if fasta is None else fasta[:fl.value]), (None if r2i is None else r2i[:rl.value])
    return out + (fo, ro) if offsets else out


def write_blocks(fd: int, buf: np.ndarray, src_off: np.ndarray, dst_off: np.ndarray, length: np.ndarray,
                 threads: int = 0) -> None:
    """pwrite block i of buf (src_off[i], length[i] bytes) at offset dst_off[i] of fd (mando_write_blocks)."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    a = [np.ascontiguousarray(x, dtype=np.int64) for x in (src_off, dst_off, length)]
    if not (len(a[0]) == len(a[1]) == len(a[2])):
        raise ValueError("write_blocks: offset and length arrays differ in length")
    if len(a[0]) and int((a[0] + a[2]).max()) > buf.size:
        raise ValueError("write_blocks: a block runs past the buffer")
    check(load().mando_write_blocks(int(fd), ptr(buf) if buf.size else None, ptr(a[0]), ptr(a[1]), ptr(a[2]),
                                    len(a[0]), threads))


class Context:
    """One mando_ctx per device (HIP stream + device buffers)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = ctypes.c_void_p()
        check(self.lib.mando_ctx_create(device, ctypes.byref(h)))
        self.handle = h
        self.device = device

    def close(self) -> None:
        if getattr(self, "handle", None):
            self.lib.mando_ctx_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self) -> None:
        check(self.lib.mando_ctx_sync(self.handle))

    def last_kernel_ms(self) -> float:
        return float(self.lib.mando_last_kernel_ms(self.handle))

    def last_kernel_launches(self) -> int:
        return int(self.lib.mando_last_kernel_launches(self.handle))

    def set_poa_budget(self, nbytes: int) -> None:
        """Explicit cap on this ctx's POA workspaces (0: the library's default policy)."""
        check(self.lib.mando_ctx_set_poa_budget(self.handle, int(nbytes)))

    def memory(self) -> tuple[int, int]:
        """(device HBM bytes, bytes held by this ctx's POA workspaces)."""
        tot, ws = ctypes.c_int64(0), ctypes.c_int64(0)
        check(self.lib.mando_ctx_memory(self.handle, ctypes.byref(tot), ctypes.byref(ws)))
        return tot.value, ws.value

    def last_slots(self) -> tuple[list[int], list[int]]:
        """Workspace slots and budgets of the last POA batch by kind (narrow, wide, -S)."""
        s, b = (ctypes.c_int64 * 3)(), (ctypes.c_int64 * 3)()
        check(self.lib.mando_poa_last_slots(self.handle, s, b))
        return list(s), list(b)

    def selftest(self) -> int:
        bad = ctypes.c_int(-1)
        check(self.lib.mando_selftest(self.handle, ctypes.byref(bad)))
        return bad.value


_ctx_cache: dict[tuple[int, int], Context] = {}


def close_contexts() -> None:
    """Destroys the cached contexts (their streams, events and device buffers).  Registered at exit: the
    library's streams each own a hardware queue, and the process should hand them back while the HIP
    runtime is still whole (a profiler that tears the runtime down first crashed on them otherwise)."""
    for c in list(_ctx_cache.values()):
        c.close()
    _ctx_cache.clear()


atexit.register(close_contexts)


def context(device: int = 0, slot: int = 0) -> Context:
    """Per-(device, slot) context: each slot owns a HIP stream and its device buffers, so two host threads
    can drive the same GPU at once (the D pipeline orients chunk k+1 on slot 1 while chunk k's POA runs
    on slot 0)."""
    c = _ctx_cache.get((device, slot))
    if c is None or c.handle is None:
        c = Context(device)
        _ctx_cache[(device, slot)] = c
    return c


def device_memory(device: int = 0) -> tuple[int, int]:
    """(free, total) HBM bytes of a device now."""
    lib = load()
    f, t = ctypes.c_int64(0), ctypes.c_int64(0)
    check(lib.mando_device_memory(int(device), ctypes.byref(f), ctypes.byref(t)))
    return f.value, t.value


def cache_trim(device: int, text_cap_max: int = -1, scratch_max: int = -1) -> int:
    """Frees the clustering's cached device buffers above the given sizes (mando_cache_trim); returns
    the bytes the caches hold afterwards."""
    lib = load()
    held = ctypes.c_int64(0)
    check(lib.mando_cache_trim(int(device), int(text_cap_max), int(scratch_max), ctypes.byref(held)))
    return held.value
