"""Synthetic R2C2 / PacBio-shaped read groups and loci (no network: the benchmark's data source).

Error model: R2C2 ~1% substitutions, 0.5% insertions, 0.5% deletions with indels
twice as likely inside homopolymers; PacBio HiFi-like 0.1% total.  Default data seed 20250117.
"""
from __future__ import annotations

import numpy as np

BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
COMP = bytes.maketrans(b"ACGTNacgtn", b"TGCANtgcan")
DATA_SEED = 20250117

R2C2 = dict(sub=0.010, ins=0.005, dele=0.005)
PACBIO = dict(sub=0.0005, ins=0.00025, dele=0.00025)


def revcomp(s: str) -> str:
    return s.encode().translate(COMP)[::-1].decode()


def random_template(rng: np.random.Generator, length: int) -> np.ndarray:
    return BASES[rng.integers(0, 4, size=length)]


def _homopolymer_mask(t: np.ndarray) -> np.ndarray:
    hp = np.zeros(len(t), dtype=bool)
    if len(t) > 1:
        same = t[1:] == t[:-1]
        hp[1:] |= same
        hp[:-1] |= same
    return hp


def mutate(rng: np.random.Generator, t: np.ndarray, sub: float, ins: float, dele: float) -> np.ndarray:
    """One noisy copy of template t (uint8 ASCII array)."""
    n = len(t)
    f = np.where(_homopolymer_mask(t), 2.0, 1.0)
    u = rng.random(n)
    pd = dele * f
    is_del = u < pd
    is_sub = (~is_del) & (u < pd + sub)
    out = t.copy()
    if is_sub.any():
        idx = np.searchsorted(BASES, out[is_sub])
        out[is_sub] = BASES[(idx + rng.integers(1, 4, size=int(is_sub.sum()))) % 4]
    is_ins = rng.random(n) < ins * f
    keep = ~is_del
    if is_ins.any():
        # insertion after position i: homopolymer extension half the time, random base otherwise
        ins_base = np.where(rng.random(n) < 0.5, t, BASES[rng.integers(0, 4, size=n)])
        ins_base = ins_base[is_ins]
        pieces_idx = np.nonzero(is_ins)[0]
        body = out.copy()
        body_keep = keep
        # assemble: kept base (if any) followed by inserted base
        counts = body_keep.astype(np.int64) + is_ins.astype(np.int64)
        res = np.empty(int(counts.sum()), dtype=np.uint8)
        starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
        kpos = starts[body_keep]
        res[kpos] = body[body_keep]
        ipos = starts[pieces_idx] + body_keep[pieces_idx].astype(np.int64)
        res[ipos] = ins_base
        return res
    return out[keep]


def read_group(rng: np.random.Generator, length: int, depth: int, model: dict = R2C2):
    """(template, reads) for one isoform: depth noisy copies of a random template of `length`."""
    t = random_template(rng, length)
    reads = [mutate(rng, t, **model).tobytes().decode() for _ in range(depth)]
    return t.tobytes().decode(), reads


def read_groups(n_groups: int, length: int | tuple[int, int], depth: int | tuple[int, int],
                seed: int = DATA_SEED, model: dict = R2C2):
    """n_groups groups; length/depth either fixed or an inclusive (lo, hi) uniform range."""
    rng = np.random.default_rng(seed)
    templates, groups = [], []
    for _ in range(n_groups):
        L = length if isinstance(length, int) else int(rng.integers(length[0], length[1] + 1))
        d = depth if isinstance(depth, int) else int(rng.integers(depth[0], depth[1] + 1))
        t, rs = read_group(rng, L, d, model)
        templates.append(t)
        groups.append(rs)
    return templates, groups
