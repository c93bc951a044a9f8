"""ctypes loader for oracle/orient_ref.c — TEST INFRASTRUCTURE ONLY (checker, never the product).

Mirrors mando_orient_batch: groups of ASCII reads (reference = the group's first read) -> per read the
strands of its primary hits.  PARITY UNPINNED vs mappy (absent from the image, see orient_ref.c).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liborient_ref.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        lib.orient_ref_batch.argtypes = [P, P, P, ctypes.c_int64, P, ctypes.c_int32, P]
        lib.orient_ref_minimizers.argtypes = [P, ctypes.c_int64, P, ctypes.c_int64]
        lib.orient_ref_minimizers.restype = ctypes.c_int64
        _lib = lib
    return _lib


def orient_batch(groups: Sequence[Sequence[str]], max_hits: int = 4) -> list[list[list[int]]]:
    lib = load()
    parts, offs, goff = [], [0], [0]
    for g in groups:
        for s in g:
            b = s.encode()
            parts.append(b)
            offs.append(offs[-1] + len(b))
        goff.append(len(offs) - 1)
    raw = np.frombuffer(b"".join(parts) or b"\0", dtype=np.uint8)
    so = np.asarray(offs, dtype=np.int64)
    go = np.asarray(goff, dtype=np.int64)
    n = len(offs) - 1
    hits = np.zeros(max(n, 1) * max_hits, dtype=np.int8)
    nh = np.zeros(max(n, 1), dtype=np.int32)
    rc = lib.orient_ref_batch(raw.ctypes.data, so.ctypes.data, go.ctypes.data, len(groups), hits.ctypes.data,
                              max_hits, nh.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"orient_ref_batch failed: {rc}")
    if n and int(nh[:n].max()) > max_hits:  # more primaries than max_hits: re-run with room for 8
        if max_hits >= 8:
            raise RuntimeError("a read has more than 8 primary hits")
        return orient_batch(groups, max_hits=8)
    out, r = [], 0
    for g in groups:
        gl = []
        for _ in g:
            gl.append([int(x) for x in hits[r * max_hits:r * max_hits + int(nh[r])]])
            r += 1
        out.append(gl)
    return out


def minimizers(s: str) -> np.ndarray:
    lib = load()
    b = np.frombuffer(s.encode() or b"\0", dtype=np.uint8)
    out = np.zeros(max(len(s), 1), dtype=np.uint64)
    n = lib.orient_ref_minimizers(b.ctypes.data, len(s), out.ctypes.data, len(out))
    return out[:max(n, 0)]


def orient_packed(seqs, seq_off, grp_off, max_hits: int = 4):
    """Packed form (mirrors mandalorion_amd.orient.orient_packed)."""
    lib = load()
    n = len(seq_off) - 1
    seqs = np.ascontiguousarray(seqs, dtype=np.uint8)
    if seqs.size == 0:
        seqs = np.zeros(1, dtype=np.uint8)
    so = np.ascontiguousarray(seq_off, dtype=np.int64)
    go = np.ascontiguousarray(grp_off, dtype=np.int64)
    hits = np.zeros((max(n, 1), max_hits), dtype=np.int8)
    nh = np.zeros(max(n, 1), dtype=np.int32)
    rc = lib.orient_ref_batch(seqs.ctypes.data, so.ctypes.data, go.ctypes.data, len(go) - 1, hits.ctypes.data,
                              max_hits, nh.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"orient_ref_batch failed: {rc}")
    return hits[:n], nh[:n]
