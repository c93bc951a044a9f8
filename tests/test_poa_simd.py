"""The cpu_baseline's vectorised POA restatement (oracle/poa_simd.c: AVX2 int16 DP rows, the scalar
restatement's graph, backtrack and consensus) is byte-identical to the scalar oracle (oracle/poa_ref.c),
DP cell counts included, on the shapes the D module hands abPOA: the edge cases, R2C2-like groups of
configs 3 / 4, deep short-read groups (many multi-predecessor rows), -S windows, and reads long enough
to take the int16 range check's scalar fallback.  CPU only."""
import numpy as np
import pytest

from mandalorion_amd import synth
from oracle import poa as opoa
from tests import poa_cases


def _same(groups, seeding=None):
    a, ca = opoa.consensus_batch(groups, return_cells=True, seeding=seeding)
    b, cb = opoa.consensus_batch(groups, return_cells=True, seeding=seeding, simd=True)
    assert a == b
    assert np.array_equal(ca, cb)
    return a


def test_edge_cases_equal_scalar():
    _same(poa_cases.edge_groups())


@pytest.mark.parametrize("length,depth,n,seed", [((300, 900), (8, 20), 12, 5), ((2000, 3600), (10, 30), 6, 7),
                                                  ((100, 300), (30, 60), 10, 3), ((4200, 5200), (6, 12), 3, 9)])
def test_noisy_groups_equal_scalar(length, depth, n, seed):
    _, groups = poa_cases.noisy_groups(n, length, depth, seed=seed)
    _same(groups)


def test_packed_config4_shape_equal_scalar():
    s, so, go = synth.fast_groups(8, (2000, 3600), (25, 25), seed=3)
    a, ao = opoa.consensus_packed(s, so, go)
    b, bo = opoa.consensus_packed(s, so, go, simd=True)
    assert np.array_equal(ao, bo) and np.array_equal(a[:ao[-1]], b[:bo[-1]])


def test_long_reads_take_the_scalar_range_fallback():
    # 6.5 kb reads: match * qlen exceeds the int16 range check, every window runs the scalar code
    s, so, go = synth.fast_groups(2, (6300, 6700), (4, 4), seed=1)
    a, ao = opoa.consensus_packed(s, so, go)
    b, bo = opoa.consensus_packed(s, so, go, simd=True)
    assert np.array_equal(ao, bo) and np.array_equal(a[:ao[-1]], b[:bo[-1]])


def test_seeded_windows_equal_scalar():
    # -S: the read is aligned window by window (align_window on subgraphs); 9 kb reads fall back per
    # window only where the window itself is too long
    _, groups = poa_cases.noisy_groups(2, (8500, 9000), (4, 5), seed=4)
    _same(groups, seeding=[True, True])
