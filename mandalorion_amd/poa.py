"""Batched partial-order-alignment consensus on the GPU (libmando `mando_poa_batch`).

Drop-in for the reference's per-isoform abPOA call
(/root/reference/utils/SpliceDefineConsensus.py:911-926): each group is the ordered list of
oriented reads that the reference would have written to `root.fasta`; the result per group is the
sequence abPOA's `-r 0` FASTA record would hold.  Unlike the reference, all groups of all loci go to
the device in one call.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from . import _lib


def pack_groups(groups: Sequence[Sequence[str | bytes]]):
    """Concatenate groups of reads into (seqs bytes, seq_off int64, grp_off int64)."""
    parts: list[bytes] = []
    lens: list[int] = []
    grp = [0]
    for g in groups:
        for s in g:
            b = s.encode() if isinstance(s, str) else bytes(s)
            parts.append(b)
            lens.append(len(b))
        grp.append(len(lens))
    seq_off = np.zeros(len(lens) + 1, dtype=np.int64)
    if lens:
        np.cumsum(np.asarray(lens, dtype=np.int64), out=seq_off[1:])
    return b"".join(parts), seq_off, np.asarray(grp, dtype=np.int64)


def poa_consensus_batch(
    groups: Sequence[Sequence[str | bytes]],
    params: _lib.PoaParams | None = None,
    seeding: Sequence[bool] | None = None,
    device: int = 0,
    return_cells: bool = False,
):
    """Consensus of every group (list of str).  Raises MandoError if the HIP path is unavailable."""
    ctx = _lib.context(device)
    p = params or _lib.PoaParams.defaults()
    seqs, seq_off, grp_off = pack_groups(groups)
    n = len(groups)
    seed_arr = None
    if seeding is not None:
        seed_arr = np.asarray([1 if s else 0 for s in seeding], dtype=np.uint8)
    cap = int(seq_off[-1]) * 2 + 1024
    cons = np.zeros(cap, dtype=np.uint8)
    cons_off = np.zeros(n + 1, dtype=np.int64)
    cells = np.zeros(max(n, 1), dtype=np.int64)
    sbuf = np.frombuffer(seqs, dtype=np.uint8) if seqs else np.zeros(1, dtype=np.uint8)
    _lib.check(
        ctx.lib.mando_poa_batch(
            ctx.handle,
            _lib.ctypes.byref(p),
            _lib.ptr(sbuf),
            _lib.ptr(seq_off),
            _lib.ptr(grp_off),
            n,
            _lib.ptr(seed_arr),
            _lib.ptr(cons),
            cap,
            _lib.ptr(cons_off),
            _lib.ptr(cells),
        )
    )
    raw = cons.tobytes()
    out = [raw[cons_off[i] : cons_off[i + 1]].decode() for i in range(n)]
    if return_cells:
        return out, cells[:n].copy()
    return out


def poa_consensus_packed(seqs: np.ndarray, seq_off: np.ndarray, grp_off: np.ndarray, seeding=None,
                         device: int = 0, params: _lib.PoaParams | None = None, info: dict | None = None,
                         slot: int = 0):
    """Packed form (no per-read Python objects): uint8 reads + int64 offsets in, consensus bytes
    (uint8) + int64 offsets (n_groups+1) out.  `info`, when given, receives the launch facts the
    roofline needs: DP cells, kernel milliseconds (HIP events on the ctx stream) and launch count.
    `slot` selects the device context (its own stream), so two host threads can keep two launches in
    flight."""
    ctx = _lib.context(device, slot)
    p = params or _lib.PoaParams.defaults()
    n = int(len(grp_off)) - 1
    seqs = np.ascontiguousarray(seqs, dtype=np.uint8)
    if seqs.size == 0:
        seqs = np.zeros(1, dtype=np.uint8)
    seq_off = np.ascontiguousarray(seq_off, dtype=np.int64)
    grp_off = np.ascontiguousarray(grp_off, dtype=np.int64)
    seed_arr = None if seeding is None else np.ascontiguousarray(np.asarray(seeding, dtype=np.uint8))
    cap = int(seq_off[-1] - seq_off[0]) * 2 + 1024
    cons = np.empty(cap, dtype=np.uint8)   # written up to cons_off[-1]; untouched pages stay unmapped
    cons_off = np.zeros(n + 1, dtype=np.int64)
    cells = np.zeros(max(n, 1), dtype=np.int64) if info is not None else None
    if n > 0:
        _lib.check(ctx.lib.mando_poa_batch(ctx.handle, _lib.ctypes.byref(p), _lib.ptr(seqs), _lib.ptr(seq_off),
                                           _lib.ptr(grp_off), n, _lib.ptr(seed_arr), _lib.ptr(cons), cap,
                                           _lib.ptr(cons_off), _lib.ptr(cells)))
        if info is not None:
            info["cells"] = int(cells[:n].sum())
            info["kernel_ms"] = ctx.last_kernel_ms()
            info["launches"] = ctx.last_kernel_launches()
    return cons[:int(cons_off[-1])], cons_off


_MADV_POPULATE_WRITE = 23  # Linux >= 5.14: fault pages in writable without changing their contents
_libc = None


def _prefault(buf: np.ndarray, nbytes: int):
    """Map the first nbytes of buf's pages in a helper thread (madvise MADV_POPULATE_WRITE; contents are
    left alone, so it may overlap writes into buf).  Returns the thread, or None."""
    global _libc
    if nbytes < (8 << 20):
        return None
    import ctypes
    import threading

    if _libc is None:
        _libc = ctypes.CDLL(None, use_errno=True)
        _libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    start = (buf.ctypes.data + 4095) & ~4095
    n = (buf.ctypes.data + nbytes - start) & ~4095
    t = threading.Thread(target=_libc.madvise, args=(start, n, _MADV_POPULATE_WRITE), daemon=True)
    t.start()
    return t


def poa_consensus_segments(d_text: int, text_len: int, off: np.ndarray, length: np.ndarray, rc: np.ndarray | None,
                           grp_off: np.ndarray, seeding=None, device: int = 0, params: _lib.PoaParams | None = None,
                           info: dict | None = None, slot: int = 0):
    """poa_consensus_packed over reads that stay on the device (mando_poa_segments): read r =
    d_text[off[r] .. off[r] + length[r]), reverse-complemented when rc[r]."""
    ctx = _lib.context(device, slot)
    p = params or _lib.PoaParams.defaults()
    n = int(len(grp_off)) - 1
    off = np.ascontiguousarray(off, dtype=np.int64)
    length = np.ascontiguousarray(length, dtype=np.int32)
    rc = None if rc is None else np.ascontiguousarray(rc, dtype=np.int8)
    grp_off = np.ascontiguousarray(grp_off, dtype=np.int64)
    seed_arr = None if seeding is None else np.ascontiguousarray(np.asarray(seeding, dtype=np.uint8))
    total = int(length.sum())
    cap = total * 2 + 1024
    cons = np.empty(cap, dtype=np.uint8)
    cons_off = np.zeros(n + 1, dtype=np.int64)
    cells = np.zeros(max(n, 1), dtype=np.int64) if info is not None else None
    if n > 0:
        # the consensi land in fresh pages of `cons` when the launch ends; faulting them in then took
        # ~20 ms per 100 MB on the path from one chunk's POA to the next, so a helper thread maps the
        # expected span (about one read per group, with margin) while the kernels run (config 4: step
        # medians 11.57 -> 11.45 s, profiles/r07d_ab_cons_prefault.txt)
        pre = _prefault(cons, min(cap, total // max(1, len(length) // n) * 5 // 4 + (1 << 20)))
        try:
            _lib.check(ctx.lib.mando_poa_segments(ctx.handle, _lib.ctypes.byref(p), _lib.ctypes.c_void_p(d_text),
                                                  int(text_len), _lib.ptr(off), _lib.ptr(length), _lib.ptr(rc),
                                                  _lib.ptr(grp_off), n, _lib.ptr(seed_arr), _lib.ptr(cons), cap,
                                                  _lib.ptr(cons_off), _lib.ptr(cells)))
        finally:
            if pre is not None:
                pre.join()
        if info is not None:
            info["cells"] = int(cells[:n].sum())
            info["kernel_ms"] = ctx.last_kernel_ms()
            info["launches"] = ctx.last_kernel_launches()
    return cons[:int(cons_off[-1])], cons_off
