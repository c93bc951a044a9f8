"""Read orientation on the GPU (libmando `mando_orient_batch`, HIP).

Drop-in for the mappy calls of determine_consensus
(/root/reference/utils/SpliceDefineConsensus.py:895-907): per isoform group, the reference is the
group's first subsampled read and every subsampled read (the first included) gets the ordered list of
strands of its primary hits.  The host then replays the reference's rebinding quirk
(mandalorion_amd.define.assemble).  Specification: oracle/orient_ref.c (parity with mappy unpinned).
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from . import _lib


def orient_batch(groups: Sequence[Sequence[str | bytes]], device: int = 0, max_hits: int = 4) -> list[list[list[int]]]:
    from .poa import pack_groups

    ctx = _lib.context(device)
    seqs, seq_off, grp_off = pack_groups(groups)
    n = int(seq_off.shape[0]) - 1
    hits = np.zeros(max(n, 1) * max_hits, dtype=np.int8)
    nh = np.zeros(max(n, 1), dtype=np.int32)
    sbuf = np.frombuffer(seqs, dtype=np.uint8) if seqs else np.zeros(1, dtype=np.uint8)
    _lib.check(ctx.lib.mando_orient_batch(ctx.handle, _lib.ptr(sbuf), _lib.ptr(seq_off), _lib.ptr(grp_off),
                                          len(groups), _lib.ptr(hits), max_hits, _lib.ptr(nh)))
    if n and int(nh[:n].max()) > max_hits:  # more primaries than max_hits: re-run with room for 8
        if max_hits >= 8:
            raise RuntimeError("a read has more than 8 primary hits")
        return orient_batch(groups, device=device, max_hits=8)
    out, r = [], 0
    for g in groups:
        gl = []
        for _ in g:
            gl.append([int(x) for x in hits[r * max_hits:r * max_hits + int(nh[r])]])
            r += 1
        out.append(gl)
    return out


def orient_packed(seqs: np.ndarray, seq_off: np.ndarray, grp_off: np.ndarray, device: int = 0, max_hits: int = 4,
                  slot: int = 0):
    """Packed form: returns (hits int8 [n_reads, max_hits], n_hits int32 [n_reads])."""
    ctx = _lib.context(device, slot)
    n = int(len(seq_off)) - 1
    seqs = np.ascontiguousarray(seqs, dtype=np.uint8)
    if seqs.size == 0:
        seqs = np.zeros(1, dtype=np.uint8)
    hits = np.zeros((max(n, 1), max_hits), dtype=np.int8)
    nh = np.zeros(max(n, 1), dtype=np.int32)
    if len(grp_off) > 1:
        _lib.check(ctx.lib.mando_orient_batch(ctx.handle, _lib.ptr(seqs), _lib.ptr(np.ascontiguousarray(seq_off, np.int64)),
                                              _lib.ptr(np.ascontiguousarray(grp_off, np.int64)), len(grp_off) - 1,
                                              _lib.ptr(hits), max_hits, _lib.ptr(nh)))
    return hits[:n], nh[:n]


def orient_segments(d_text: int, text_len: int, off: np.ndarray, length: np.ndarray, grp_off: np.ndarray,
                    device: int = 0, max_hits: int = 4, slot: int = 0):
    """orient_packed over reads that stay on the device: read r = d_text[off[r] .. off[r] + length[r])
    (mando_orient_segments; d_text from ClusterResult.device_text())."""
    ctx = _lib.context(device, slot)
    n = int(len(off))
    off = np.ascontiguousarray(off, dtype=np.int64)
    length = np.ascontiguousarray(length, dtype=np.int32)
    hits = np.zeros((max(n, 1), max_hits), dtype=np.int8)
    nh = np.zeros(max(n, 1), dtype=np.int32)
    if len(grp_off) > 1:
        _lib.check(ctx.lib.mando_orient_segments(ctx.handle, _lib.ctypes.c_void_p(d_text), int(text_len), _lib.ptr(off),
                                                 _lib.ptr(length), _lib.ptr(np.ascontiguousarray(grp_off, np.int64)),
                                                 len(grp_off) - 1, _lib.ptr(hits), max_hits, _lib.ptr(nh)))
    return hits[:n], nh[:n]
