"""The wide groups of a chunk as a batch of their own (define.py _WIDE_SLOT): the split restates the
library's launch rule (capi.hip poa_batch_impl: abPOA's adaptive band at the group's mean read length,
wide past 116 columns, -S groups apart), and the subset batches carry exactly their groups' reads."""
import numpy as np
import pytest

from mandalorion_amd import define


def _ref_wide(length, grp_off, seeding):
    out = []
    for g in range(len(grp_off) - 1):
        lens = [int(x) for x in length[grp_off[g]:grp_off[g + 1]]]
        mean = sum(lens) // max(1, len(lens))
        w = 10 + int(np.float32(0.01) * np.float32(mean))
        out.append(bool(2 * w + 1 > 116 and not seeding[g]))
    return np.array(out)


def test_wide_groups_restate_the_launch_rule():
    rng = np.random.default_rng(4)
    n = 500
    counts = rng.integers(0, 30, size=n)
    grp_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    length = rng.integers(0, 9000, size=int(grp_off[-1])).astype(np.int32)
    seeding = (rng.random(n) < 0.1).astype(np.uint8)
    got = define._wide_groups(length, grp_off, seeding)
    assert np.array_equal(got, _ref_wide(length, grp_off, seeding))
    assert got.any() and not got.all()
    # the band edge: a mean of 4799 is narrow (w = 57), 4800 wide (w = 58)
    g = np.array([0, 1, 2], dtype=np.int64)
    assert list(define._wide_groups(np.array([4799, 4800], np.int32), g, None)) == [False, True]


def test_group_subset_keeps_each_groups_reads():
    rng = np.random.default_rng(5)
    counts = rng.integers(0, 6, size=50)
    grp_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    nr = int(grp_off[-1])
    off = rng.integers(0, 1 << 30, size=nr).astype(np.int64)
    length = rng.integers(1, 5000, size=nr).astype(np.int32)
    rc = rng.integers(0, 2, size=nr).astype(np.int8)
    seeding = rng.integers(0, 2, size=50).astype(np.uint8)
    mask = rng.random(50) < 0.4
    gidx, o2, l2, r2, g2, s2 = define._group_subset(off, length, rc, grp_off, seeding, mask)
    assert np.array_equal(gidx, np.flatnonzero(mask))
    assert np.array_equal(s2, seeding[mask])
    for k, g in enumerate(gidx):
        a, b = grp_off[g], grp_off[g + 1]
        c, d = g2[k], g2[k + 1]
        assert np.array_equal(o2[c:d], off[a:b]) and np.array_equal(l2[c:d], length[a:b])
        assert np.array_equal(r2[c:d], rc[a:b])


@pytest.mark.gpu
def test_define_gpu_split_wide_equals_one_batch(gpu_ctx, tmp_path, monkeypatch):
    """Three chunks with the wide groups on their own context and thread, against the same chunks with the
    wide groups in the chunk's batch: same files."""
    from tests.test_define_gpu import _run
    from mandalorion_amd import synth

    d = str(tmp_path)
    # 2-10 kb reads: groups on both sides of the wide band (mean read length ~4.8 kb)
    synth.write_loci(f"{d}/tmp_SS", 90, reads=(12, 30), exons=(8, 14), exon_len=(250, 700), seed=21, rev_frac=0.5)
    read = lambda f: open(f"{d}/{f}", "rb").read()  # noqa: E731
    monkeypatch.setattr(define, "_SPLIT_WIDE", False)
    st0 = _run(d, "None", n_chunks=3)
    ref = read("Isoform_Consensi.fasta"), read("reads2isoforms.txt")
    monkeypatch.setattr(define, "_SPLIT_WIDE", True)
    st1 = _run(d, "None", n_chunks=3)
    assert st0["split_wide_groups"] == 0 and st1["split_wide_groups"] > 0
    assert len(st1["poa_launches"]) == 3
    assert (read("Isoform_Consensi.fasta"), read("reads2isoforms.txt")) == ref
