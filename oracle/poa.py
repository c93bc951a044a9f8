"""ctypes loader for oracle/poa_ref.c — TEST INFRASTRUCTURE ONLY (checker, never the product).

Mirrors mando_poa_batch: groups of ASCII reads in abPOA input order -> consensus strings + DP cell
counts.  Builds oracle/build/libpoa_ref.so with `make -C oracle` when it is missing.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libpoa_ref.so")
# the same restatement with AVX2 int16 DP rows (poa_simd.c): bench.py's cpu_baseline, byte-equal to LIB
LIB_SIMD = os.path.join(HERE, "build", "libpoa_simd.so")


class Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("match", "mismatch", "gap_open1", "gap_ext1", "gap_open2", "gap_ext2", "band_b")] + \
               [("band_f", ctypes.c_float)] + \
               [(n, ctypes.c_int32) for n in ("seeding", "k", "w", "min_w")]

    @classmethod
    def defaults(cls) -> "Params":
        return cls(5, 4, 4, 2, 24, 1, 10, 0.01, 0, 19, 10, 500)


_libs: dict = {}


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def load(simd: bool = False):
    path = LIB_SIMD if simd else LIB
    if path not in _libs:
        if not os.path.exists(path):
            build()
        lib = ctypes.CDLL(path)
        P = ctypes.c_void_p
        lib.poa_ref_batch.argtypes = [P, P, P, P, ctypes.c_int64, P, P, ctypes.c_int64, P, P]
        lib.poa_ref_batch.restype = ctypes.c_int
        lib.poa_ref_seed_partition.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, P, P, ctypes.c_int]
        lib.poa_ref_seed_partition.restype = ctypes.c_int
        _libs[path] = lib
    return _libs[path]


_ENC = np.full(256, 4, dtype=np.uint8)
for _c, _v in zip(b"ACGTacgt", (0, 1, 2, 3, 0, 1, 2, 3)):
    _ENC[_c] = _v


def seed_partition(t: str, q: str, params: Params | None = None) -> list[tuple[int, int]]:
    """-S partition anchors (k-mer starts in t, in q) of read q against the previous read t."""
    lib = load()
    p = params or Params.defaults()
    te = _ENC[np.frombuffer(t.encode() or b"N", dtype=np.uint8)]
    qe = _ENC[np.frombuffer(q.encode() or b"N", dtype=np.uint8)]
    cap = len(q) // max(1, p.min_w) + 2
    pt = np.zeros(cap, dtype=np.int32)
    pq = np.zeros(cap, dtype=np.int32)
    n = lib.poa_ref_seed_partition(te.ctypes.data, len(t), qe.ctypes.data, len(q), p.k, p.w, p.min_w,
                                   pt.ctypes.data, pq.ctypes.data, cap)
    return list(zip(pt[:n].tolist(), pq[:n].tolist()))


def consensus_batch(groups: Sequence[Sequence[str]], params: Params | None = None,
                    return_cells: bool = False, seeding: Sequence[bool] | None = None, simd: bool = False):
    lib = load(simd)
    p = params or Params.defaults()
    parts, lens, grp = [], [], [0]
    for g in groups:
        for s in g:
            b = s.encode() if isinstance(s, str) else bytes(s)
            parts.append(b)
            lens.append(len(b))
        grp.append(len(lens))
    seqs = np.frombuffer(b"".join(parts) or b"\0", dtype=np.uint8)
    seq_off = np.zeros(len(lens) + 1, dtype=np.int64)
    if lens:
        np.cumsum(lens, out=seq_off[1:])
    grp_off = np.asarray(grp, dtype=np.int64)
    n = len(groups)
    cap = int(seq_off[-1]) * 2 + 1024
    out = np.zeros(cap, dtype=np.uint8)
    cons_off = np.zeros(n + 1, dtype=np.int64)
    cells = np.zeros(max(n, 1), dtype=np.int64)
    sd = None if seeding is None else np.asarray([1 if x else 0 for x in seeding], dtype=np.uint8)
    rc = lib.poa_ref_batch(ctypes.addressof(p), seqs.ctypes.data, seq_off.ctypes.data,
                           grp_off.ctypes.data, n, None if sd is None else sd.ctypes.data, out.ctypes.data, cap,
                           cons_off.ctypes.data, cells.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"poa_ref_batch failed: {rc}")
    raw = out.tobytes()
    cons = [raw[cons_off[i]:cons_off[i + 1]].decode() for i in range(n)]
    return (cons, cells[:n].copy()) if return_cells else cons


def consensus_packed(seqs, seq_off, grp_off, params: Params | None = None, seeding=None, simd: bool = False,
                     cells_out=None):
    """Packed form of consensus_batch (mirrors mandalorion_amd.poa.poa_consensus_packed); cells_out (an
    int64 array of one entry per group, optional) receives the DP cell counts."""
    lib = load(simd)
    p = params or Params.defaults()
    seqs = np.ascontiguousarray(seqs, dtype=np.uint8)
    if seqs.size == 0:
        seqs = np.zeros(1, dtype=np.uint8)
    seq_off = np.ascontiguousarray(seq_off, dtype=np.int64)
    grp_off = np.ascontiguousarray(grp_off, dtype=np.int64)
    n = len(grp_off) - 1
    cap = int(seq_off[-1] - seq_off[0]) * 2 + 1024
    out = np.zeros(cap, dtype=np.uint8)
    cons_off = np.zeros(n + 1, dtype=np.int64)
    sd = None if seeding is None else np.ascontiguousarray(np.asarray(seeding, dtype=np.uint8))
    if n > 0:
        rc = lib.poa_ref_batch(ctypes.addressof(p), seqs.ctypes.data, seq_off.ctypes.data, grp_off.ctypes.data, n,
                               None if sd is None else sd.ctypes.data, out.ctypes.data, cap, cons_off.ctypes.data,
                               None if cells_out is None else cells_out.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"poa_ref_batch failed: {rc}")
    return out, cons_off
