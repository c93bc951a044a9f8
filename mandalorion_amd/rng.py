"""Seeded replay of the reference's subsampling draws (libmando `mando_mt_permutation`).

Every locus worker in the reference is forked from one parent RNG state
(/root/reference/defineIsoforms.py:130), so each locus consumes the stream of a fresh legacy
`RandomState(seed)`: draws at SpliceDefineConsensus.py:505 (characterize_splicing_event, k=500),
:818 (define_start_end_sites, k=10000) and :884 (determine_consensus, k=100), in that call order.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from . import _lib


def permutation_draws(seed: int, draws: Sequence[tuple[int, int]]) -> list[np.ndarray]:
    """[(n, k), ...] -> [RandomState(seed) choice(arange(n), k, replace=False) for each, in order]."""
    ns = np.asarray([d[0] for d in draws], dtype=np.int64)
    ks = np.asarray([min(d[0], d[1]) for d in draws], dtype=np.int64)
    total = int(ks.sum()) if len(ks) else 0
    out = np.zeros(max(total, 1), dtype=np.int64)
    lib = _lib.load()
    _lib.check(lib.mando_mt_permutation(seed & 0xFFFFFFFF, _lib.ptr(ns), _lib.ptr(ks), len(ns),
                                        _lib.ptr(out), total))
    res, o = [], 0
    for k in ks:
        res.append(out[o:o + k].copy())
        o += int(k)
    return res
