"""Orientation: the HIP kernel vs the CPU restatement (oracle/orient_ref.c), and both vs the true strand
of synthetic reads.  PARITY UNPINNED against mappy (absent; no reference test or fixture exists for this
step) — the GPU/CPU comparison is bit-exact on the full hit lists."""
from __future__ import annotations

import numpy as np
import pytest

from mandalorion_amd import synth


def _groups(n_groups, seed, flip_p=0.3, lens=(2500, 3500), depth=(5, 30), unrelated=True):
    _, groups = synth.read_groups(n_groups, lens, depth, seed=seed)
    rng = np.random.default_rng(seed + 100)
    out, truth = [], []
    for g in groups:
        f = [bool(rng.random() < flip_p) and i > 0 for i in range(len(g))]
        gg = [synth.revcomp(s) if x else s for s, x in zip(g, f)]
        t = [[-1] if x else [1] for x in f]
        if unrelated:
            gg.append("".join(rng.choice(list("ACGT"), int(rng.integers(500, 3000)))))
            t.append([])
        out.append(gg)
        truth.append(t)
    return out, truth


def test_oracle_recovers_true_strand():
    from oracle import orient as oref

    groups, truth = _groups(12, 5)
    assert oref.orient_batch(groups) == truth


def test_oracle_edge_cases():
    from oracle import orient as oref

    short = ["ACGT", "ACGTACGTAC", "N" * 50]
    g = [["ACGTTGCA" * 40] + short, short]
    res = oref.orient_batch(g)
    assert res[0][1:] == [[], [], []]
    assert res[1] == [[], [], []]


def _chimera_group():
    """A query made of the reference's two halves, the second one reverse-complemented: two primary
    hits (one per strand), which the reference writes twice (SpliceDefineConsensus.py:902-907)."""
    rng = np.random.default_rng(41)
    a = "".join(rng.choice(list("ACGT"), 1500))
    b = "".join(rng.choice(list("ACGT"), 1500))
    return [a + b, a + synth.revcomp(b), a + b]


def test_oracle_counts_primaries_past_max_hits():
    from oracle import orient as oref

    g = [_chimera_group()]
    lib = oref.load()
    raw = "".join(g[0]).encode()
    so = np.cumsum([0] + [len(s) for s in g[0]]).astype(np.int64)
    go = np.array([0, 3], dtype=np.int64)
    hits = np.zeros(3, dtype=np.int8)
    nh = np.zeros(3, dtype=np.int32)
    buf = np.frombuffer(raw, dtype=np.uint8)
    assert lib.orient_ref_batch(buf.ctypes.data, so.ctypes.data, go.ctypes.data, 1, hits.ctypes.data, 1,
                                nh.ctypes.data) == 0
    assert nh.tolist() == [1, 2, 1]  # 2 = max_hits + 1: overflow reported, not truncated
    res = oref.orient_batch(g, max_hits=1)  # re-run with room for 8
    assert sorted(res[0][1]) == [-1, 1] and res[0][0] == [1] and res[0][2] == [1]


@pytest.mark.gpu
def test_orient_gpu_reports_extra_primaries(gpu_ctx):
    from mandalorion_amd import orient
    from oracle import orient as oref

    g = [_chimera_group()] + _groups(5, 3)[0]
    assert orient.orient_batch(g, max_hits=1) == oref.orient_batch(g, max_hits=1)
    assert sorted(orient.orient_batch(g, max_hits=1)[0][1]) == [-1, 1]


@pytest.mark.gpu
def test_orient_gpu_matches_oracle(gpu_ctx):
    from mandalorion_amd import orient
    from oracle import orient as oref

    groups, truth = _groups(40, 11)
    groups += _groups(10, 12, lens=(300, 900), depth=(2, 6))[0]
    groups += [["ACGT", "A" * 40, "ACGTACGTACGTACGTAC"], ["N" * 100, "ACGTTGCA" * 30]]
    got = orient.orient_batch(groups)
    assert got == oref.orient_batch(groups)
    assert got[:40] == truth


@pytest.mark.gpu
def test_orient_gpu_long_reads(gpu_ctx):
    from mandalorion_amd import orient
    from oracle import orient as oref

    groups, truth = _groups(6, 21, lens=(7000, 9000), depth=(5, 12))
    got = orient.orient_batch(groups)
    assert got == oref.orient_batch(groups) == truth


@pytest.mark.gpu
def test_orient_gpu_capacity_rerun(gpu_ctx):
    """A 3-copy tandem repeat gives ~3 anchors per query minimizer: over the first launch's per-read
    capacity (1024 for these lengths), so the host re-runs that group at 2048; the other groups of the
    batch keep their first-launch results.  Same hit lists as the restatement."""
    from mandalorion_amd import orient
    from oracle import orient as oref

    rng = np.random.default_rng(31)
    unit = "".join(rng.choice(list("ACGT"), 1000))
    rep = [unit * 3, unit * 3, synth.revcomp(unit * 3), unit[:500] + unit * 2]
    groups, _ = _groups(20, 33)
    groups = groups[:10] + [rep] + groups[10:]
    got = orient.orient_batch(groups)
    assert got == oref.orient_batch(groups)
    assert got[10][1] == [1] and got[10][2] == [-1]


@pytest.mark.gpu
def test_orient_gpu_reads_beyond_lds_capacity(gpu_ctx):
    """Reads of 20-40 kb hold more minimizers than the LDS capacity (2048): those groups re-run with
    the arrays in per-wave HBM slabs instead of being refused (mappy has no such limit).  Same hit
    lists as the restatement, and the true strands; short groups in the same batch are unaffected."""
    from mandalorion_amd import orient
    from oracle import orient as oref

    long_groups, long_truth = _groups(3, 41, lens=(20000, 40000), depth=(3, 5))
    short_groups, short_truth = _groups(8, 42)
    groups = short_groups[:4] + long_groups + short_groups[4:]
    truth = short_truth[:4] + long_truth + short_truth[4:]
    got = orient.orient_batch(groups)
    assert got == oref.orient_batch(groups) == truth


@pytest.mark.gpu
def test_orient_gpu_more_groups_than_waves(gpu_ctx):
    """More groups than the launch has waves (4,096 on MI355X at 16 per CU), so every wave reuses its HBM
    slab of reference keys for several groups: same hit lists as the restatement."""
    from mandalorion_amd import orient
    from oracle import orient as oref

    groups, truth = _groups(9000, 61, lens=(300, 700), depth=(2, 4), unrelated=False)
    got = orient.orient_batch(groups)
    assert got == oref.orient_batch(groups)
    assert got == truth
