"""Per-locus read clustering on the GPU (libmando `mando_cluster_loci`: host threads read the locus
files, two HIP kernels cluster one locus per wave, csrc/cluster_kernel.hip).

Replaces the clustering half of the reference's `process_locus`
(/root/reference/defineIsoforms.py:55-91: collect_reads, make_genome_bins, find_peaks,
sort_reads_into_splice_junctions, define_start_end_sites) plus the subsample draw of
`determine_consensus` (/root/reference/utils/SpliceDefineConsensus.py:884-888).  Each locus replays the
numpy RNG stream of `RandomState(seed)`, i.e. what every forked locus worker of the reference sees when
the parent seeded numpy before `mp.Pool` (defineIsoforms.py:130).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib

STATUS = {0: "ok", -10: "ZeroDivisionError", -11: "KeyError", -12: "parse error", -13: "I/O error",
          -14: "IndexError", -15: "ValueError"}


@dataclass
class Peak:
    start: int
    end: int
    type: str
    side: str
    prop: float  # -1.0 for annotated bins ('A')

    @property
    def prop_str(self) -> str:
        """str(proportion) as the reference writes it (toWrite[5])."""
        return "A" if self.prop < 0 else repr(float(self.prop))


def _arr(p, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(p, shape=(n,)).copy()


class ClusterResult:
    """Owns a mando_cluster_result; arrays are copied out, the text buffer is viewed in place.
    view_get / free default to libmando's (the oracle passes its own)."""

    def __init__(self, handle: ctypes.c_void_p, view_get=None, free=None):
        self._lib = _lib.load()
        self._h = handle
        self._free = free or self._lib.mando_cluster_free
        self.on_close = None  # called once, when the result's buffers are released
        v = _lib.ClusterView()
        _lib.check((view_get or self._lib.mando_cluster_view_get)(handle, ctypes.byref(v)))
        self.n_loci = v.n_loci
        self.n_records = v.n_records
        self.locus_status = _arr(v.locus_status, v.n_loci, np.int32)
        self.text = (np.ctypeslib.as_array(ctypes.cast(v.text, ctypes.POINTER(ctypes.c_uint8)), shape=(v.text_len,))
                     if v.text_len else np.zeros(0, dtype=np.uint8))
        n = v.n_records
        self.name_off = _arr(v.name_off, n, np.int64)
        self.name_len = _arr(v.name_len, n, np.int32)
        self.seq_off = _arr(v.seq_off, n, np.int64)
        self.seq_len = _arr(v.seq_len, n, np.int32)
        self.rec_locus = _arr(v.rec_locus, n, np.int64)
        ni = v.n_isoforms
        self.iso_locus = _arr(v.iso_locus, ni, np.int64)
        self.mem_off = _arr(v.mem_off, ni + 1, np.int64)
        self.mem = _arr(v.mem, int(self.mem_off[-1]), np.int64)
        self.sub_off = _arr(v.sub_off, ni + 1, np.int64)
        self.sub = _arr(v.sub, int(self.sub_off[-1]), np.int64)
        npk = v.n_peaks
        self.peak_locus = _arr(v.peak_locus, npk, np.int64)
        self.peak_start = _arr(v.peak_start, npk, np.int64)
        self.peak_end = _arr(v.peak_end, npk, np.int64)
        self.peak_type = bytes(_arr(v.peak_type, npk, np.uint8)).decode() if npk else ""
        self.peak_side = bytes(_arr(v.peak_side, npk, np.uint8)).decode() if npk else ""
        self.peak_prop = _arr(v.peak_prop, npk, np.float64)
        # the subsampled reads' orientation, when the call ran it (orient=True): sub x H hit strands
        H = int(getattr(v, "orient_max_hits", 0) or 0)
        self.orient_hits = self.orient_n_hits = None
        if H > 0:
            ns = int(self.sub_off[-1])
            self.orient_hits = _arr(v.orient_hits, ns * H, np.int8).reshape(ns, H)
            self.orient_n_hits = _arr(v.orient_n_hits, ns, np.int32)

    def device_text(self) -> tuple[int, int]:
        """(device pointer, length) of the locus text on the GPU the clustering ran on (0 for the
        restatement's results, which have none)."""
        if not hasattr(self._lib, "mando_cluster_device_text") or self._free != self._lib.mando_cluster_free:
            return 0, 0
        d = ctypes.c_void_p()
        n = ctypes.c_int64()
        _lib.check(self._lib.mando_cluster_device_text(self._h, ctypes.byref(d), ctypes.byref(n)))
        return int(d.value or 0), int(n.value)

    def close(self):
        if self._h is not None:
            self._free(self._h)
            self._h = None
            self.text = np.zeros(0, dtype=np.uint8)
            cb, self.on_close = self.on_close, None
            if cb is not None:
                cb()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def n_isoforms(self) -> int:
        return len(self.iso_locus)

    def name(self, r: int) -> str:
        a = int(self.name_off[r])
        return bytes(self.text[a:a + int(self.name_len[r])]).decode()

    def seq(self, r: int) -> str:
        a = int(self.seq_off[r])
        return bytes(self.text[a:a + int(self.seq_len[r])]).decode()

    def members(self, i: int) -> np.ndarray:
        return self.mem[self.mem_off[i]:self.mem_off[i + 1]]

    def subsample(self, i: int) -> np.ndarray:
        return self.sub[self.sub_off[i]:self.sub_off[i + 1]]

    def peaks(self, locus: int) -> list[Peak]:
        idx = np.nonzero(self.peak_locus == locus)[0]
        return [Peak(int(self.peak_start[k]), int(self.peak_end[k]), self.peak_type[k], self.peak_side[k],
                     float(self.peak_prop[k])) for k in idx]


def cluster_params(cutoff: float = 0.1, splice_site_width: int = 1, minimum_read_count: int = 2,
                   upstream_buffer: int = 10, downstream_buffer: int = 50,
                   junctions: str = "gtag,gcag,atac,ctac,ctgc,gtat", seed: int = 0, threads: int = 0,
                   poa_subsample: int = 100):
    p = _lib.ClusterParams()
    _lib.load().mando_cluster_default_params(ctypes.byref(p))
    p.cutoff = cutoff
    p.splice_site_width = splice_site_width
    p.minimum_read_count = minimum_read_count
    p.upstream_buffer = upstream_buffer
    p.downstream_buffer = downstream_buffer
    p.junctions = junctions.encode()  # ctypes keeps the bytes alive with the struct
    p.seed = seed & 0xFFFFFFFF
    p.threads = threads
    p.poa_subsample = poa_subsample
    return p


def c_inputs(paths: list[str], chroms: list[str], ann):
    """ctypes arrays of the locus paths / chroms and the flattened annotated bounds."""
    n = len(paths)
    cpaths = (ctypes.c_char_p * max(n, 1))(*[x.encode() for x in paths])
    cchroms = (ctypes.c_char_p * max(n, 1))(*[x.encode() for x in chroms])
    ann_pos = ann_off = None
    if ann is not None:
        parts = [np.asarray(ann[i][s], dtype=np.int64).ravel() for i in range(n) for s in range(4)]
        off = np.zeros(4 * n + 1, dtype=np.int64)
        np.cumsum([len(x) for x in parts], out=off[1:])
        ann_pos = np.concatenate(parts) if parts and off[-1] else np.zeros(1, dtype=np.int64)
        ann_off = off
    return n, cpaths, cchroms, ann_pos, ann_off


def cluster_loci(paths: list[str], chroms: list[str], ann: list[list[list[int]]] | None = None,
                 device: int = 0, slot: int = 4, orient: bool = False, **params) -> ClusterResult:
    """Cluster every locus file on the GPU.  ann[i] = [left '5', left '3', right '5', right '3'] position
    lists; params as cluster_params (threads: host threads reading the files).  orient: every isoform's
    subsample is also oriented (on the device's orientation context, slot 1) as its loci are clustered;
    the result then holds orient_hits / orient_n_hits (None when a read had more than 8 primary hits)."""
    lib = _lib.load()
    p = cluster_params(**params)
    if orient:
        p.orient_ctx = _lib.context(device, slot=1).handle.value
    n, cpaths, cchroms, ann_pos, ann_off = c_inputs(paths, chroms, ann)
    ctx = _lib.context(device, slot=slot)
    h = ctypes.c_void_p()
    _lib.check(lib.mando_cluster_loci(ctx.handle, ctypes.byref(p), cpaths, cchroms, n, _lib.ptr(ann_pos),
                                      _lib.ptr(ann_off), ctypes.byref(h)))
    return ClusterResult(h)
