"""HIP POA kernel == CPU restatement (oracle/poa_ref.c), byte for byte, plus identical DP cell counts.

Runs through the C-ABI (libmando mando_poa_batch).  Exact equality is the bar: consensus bytes are
integer/index work."""
import numpy as np
import pytest

from mandalorion_amd import poa, synth
from oracle import poa as opoa
from tests import poa_cases

pytestmark = pytest.mark.gpu


def _check(groups, seeding=None):
    got, gcells = poa.poa_consensus_batch(groups, return_cells=True, seeding=seeding)
    want, wcells = opoa.consensus_batch(groups, return_cells=True, seeding=seeding)
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert not bad, f"{len(bad)} groups differ, first {bad[:5]}"
    assert np.array_equal(gcells, wcells)
    return got


def test_wave_primitives_selftest(gpu_ctx):
    assert gpu_ctx.selftest() == 0


def test_edge_cases_match_oracle():
    _check(poa_cases.edge_groups())


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_small_noisy_groups_match_oracle(seed):
    _check(poa_cases.noisy_groups(40, (50, 700), (2, 25), seed=seed)[1])


def test_r2c2_3kb_groups_match_oracle():
    _check(poa_cases.noisy_groups(24, (2000, 4000), (10, 30), seed=77)[1])


def test_pacbio_like_and_noisy_mix():
    _, a = synth.read_groups(8, (1000, 2500), (5, 15), seed=4, model=synth.PACBIO)
    _, b = synth.read_groups(8, (500, 1500), (5, 15), seed=5, model=dict(sub=0.04, ins=0.03, dele=0.03))
    _check(a + b)


def test_many_groups_one_launch_is_order_independent():
    _, groups = poa_cases.noisy_groups(300, (100, 400), (3, 8), seed=123)
    full = poa.poa_consensus_batch(groups)
    part = poa.poa_consensus_batch(groups[::-1])[::-1]
    assert full == part
    want = opoa.consensus_batch(groups)
    assert full == want


def test_wide_band_and_far_predecessors():
    rng = np.random.default_rng(8)
    t = synth.random_template(rng, 1500).tobytes().decode()
    ins = synth.random_template(rng, 300).tobytes().decode()
    groups = [[t, t[:700] + ins + t[700:], t, t[:400] + t[700:], t[:700] + ins + t[700:], t]]
    _check(groups)


def test_long_reads_beyond_8kb():
    """Reads of 8-12 kb (config-5 lengths; the read buffer is sized per batch in dynamic LDS)."""
    _check(poa_cases.noisy_groups(4, (8000, 12000), (4, 8), seed=31)[1])


def test_mixed_lengths_one_batch():
    """Short and long groups in one launch: LDS sizing and occupancy follow the longest read."""
    _, a = poa_cases.noisy_groups(30, (200, 900), (3, 10), seed=41)
    _, b = poa_cases.noisy_groups(2, (9000, 10000), (3, 5), seed=42)
    _check(a + b)


def test_config5_deep_long_group():
    """Config-5 shape: one isoform of 100 reads x ~8.5 kb, run through the -S path the reference takes
    for it (median length >= 8000 -> `abpoa -S`, SpliceDefineConsensus.py:915-919): seed kernel
    partition + window DPs, byte-equal to the oracle's -S restatement, with far fewer DP cells than
    the unseeded alignment of the same group."""
    g = poa_cases.noisy_groups(1, (8300, 8700), (100, 100), seed=55)[1]
    _, seeded_cells = opoa.consensus_batch(g, return_cells=True, seeding=[1])
    _, full_cells = opoa.consensus_batch(g, return_cells=True)
    assert seeded_cells[0] < full_cells[0] / 3  # the seeded path ran (windows, not one 8.5 kb band)
    _check(g, seeding=[1])


def test_seeded_groups_mixed_with_unseeded():
    """-S and plain groups in one call (two launches: the seeded and unseeded kernel instantiations),
    short seeded groups (no anchors: plain DP), N runs, and a read sharing no k-mer with its
    predecessor (one window)."""
    _, long_g = poa_cases.noisy_groups(6, (5000, 9000), (4, 12), seed=61)
    _, short_g = poa_cases.noisy_groups(6, (200, 900), (3, 8), seed=62)
    rng = np.random.default_rng(63)
    t = synth.random_template(rng, 4000).tobytes().decode()
    u = synth.random_template(rng, 3000).tobytes().decode()
    odd = [[t, t[:1500] + "N" * 40 + t[1540:], u, t, t[:2000] + t[2100:]]]
    groups = long_g + short_g + odd + long_g[:2]
    seeding = [1] * 6 + [1, 0, 1, 0, 1, 0] + [1] + [0, 0]
    _check(groups, seeding=seeding)


@pytest.mark.parametrize("persistent", [False, True])
def test_grid_modes_and_launch_kinds(gpu_ctx, persistent):
    """One-group grids (a workgroup per group, workspace slots claimed from a flag array) and the
    persistent grid (fewer slots than groups: a 128 MiB workspace budget) give the same consensi; the batch
    spans the narrow (3 kb), wide (6-9 kb: 256-column ring rows, 16-bit mode shifted past 6.4 kb) and
    32-bit wide (> 10.1 kb) launch kinds at once."""
    from mandalorion_amd import _lib

    _, narrow = poa_cases.noisy_groups(40, (2700, 3300), (4, 12), seed=81)
    _, wide = poa_cases.noisy_groups(4, (6000, 9000), (4, 10), seed=82)
    _, longer = poa_cases.noisy_groups(2, (10500, 11500), (3, 5), seed=83)
    ctx = _lib.context(0, 0)
    ctx.set_poa_budget((128 << 20) if persistent else 0)
    try:
        _check(narrow + wide + longer)
        if persistent:
            slots, _ = ctx.last_slots()
            assert 0 < slots[0] < 40  # the narrow launch ran fewer slots than groups: the persistent grid
    finally:
        ctx.set_poa_budget(0)


def test_narrow_groups_at_the_band_threshold(gpu_ctx):
    """Mean reads of 4.5-5.0 kb: bands 2w + 1 of 111-121 columns, on both sides of the narrow / wide split
    (kWideBand); the narrow ones (113, 115) run rows of one chunk whose drift past 128 columns takes the
    generic row and its HBM spill.  Same consensi as the restatement."""
    _, groups = poa_cases.noisy_groups(12, (4500, 5000), (4, 8), seed=84)
    _check(groups)


@pytest.mark.parametrize("waves", ["0", "2"])
def test_wide_launch_waves_per_group(monkeypatch, waves):
    """Wide launches with one or two waves per group (MANDO_POA_W2=0: one wave; 2, the default: every
    two-chunk fast row split over
    the two waves of the group's workgroup, poa_kernel.hip row16w_half; one-chunk, generic and 32-bit rows
    stay on wave 0): the same bytes and DP cells as the oracle.  The batch spans bands just over one chunk
    (5-6 kb), two full chunks (8-9 kb, 16-bit shifted), 32-bit rows (> 10.1 kb), deep and shallow groups,
    and rows with several predecessors (indels shared by several reads)."""
    monkeypatch.setenv("MANDO_POA_W2", waves)
    _, mid = poa_cases.noisy_groups(6, (5000, 6000), (6, 30), seed=91)
    _, long_g = poa_cases.noisy_groups(3, (8000, 9000), (4, 12), seed=92)
    _, longer = poa_cases.noisy_groups(1, (10500, 11000), (3, 4), seed=93)
    rng = np.random.default_rng(94)
    t = synth.random_template(rng, 6000).tobytes().decode()
    ins = synth.random_template(rng, 300).tobytes().decode()
    branchy = [[t, t[:2500] + ins + t[2500:], t, t[:2000] + t[2600:], t[:2500] + ins + t[2500:], t[:4000] + "N" * 30 + t[4030:], t]]
    _check(mid + long_g + longer + branchy)


def test_wide_two_waves_deep_long_group(monkeypatch):
    """Config-5's unseeded shape (one wave per group is its critical path): 40 reads x ~8.5 kb, two waves."""
    monkeypatch.setenv("MANDO_POA_W2", "2")
    _check(poa_cases.noisy_groups(1, (8300, 8700), (40, 40), seed=95)[1])


@pytest.mark.parametrize("team", ["1", "3", "8"])
def test_seeded_team_sizes(monkeypatch, team):
    """-S teams (poa_kernel.hip "-S teams"): a read's windows aligned by 1 (solo), 3 or 8 workgroups
    give the same consensi; 10 seeded groups share the launch with two unseeded ones."""
    monkeypatch.setenv("MANDO_TEAM", team)
    _, long_g = poa_cases.noisy_groups(10, (7000, 9000), (6, 14), seed=71)
    _, short_g = poa_cases.noisy_groups(2, (500, 900), (3, 6), seed=72)
    _check(long_g + short_g, seeding=[1] * 10 + [0, 0])


def test_seeded_32bit_rows(monkeypatch):
    monkeypatch.setenv("MANDO_POA_DBG", "1")
    _check(poa_cases.noisy_groups(3, (6000, 8000), (5, 10), seed=64)[1], seeding=[1, 1, 1])


def test_config3_full_size_properties():
    """BASELINE config 3 at full size per GPU is 20k groups; here 2k of them through the same launch
    path, checked by size-independent properties: every consensus is non-empty ACGT, within 10 % of
    the template length, and 50 strided groups match the CPU restatement byte for byte."""
    import numpy as np
    seqs, so, go, tmpl = synth.fast_groups(2000, (2700, 3300), (50, 50), seed=2025, threads=8, with_templates=True)
    groups = synth.unpack_groups(seqs, so, go)
    got = poa.poa_consensus_batch(groups)
    assert all(g and set(g) <= set("ACGT") for g in got)
    ratio = np.array([len(g) / len(t) for g, t in zip(got, tmpl)])
    assert ratio.min() > 0.9 and ratio.max() < 1.1
    pick = list(range(0, 2000, 40))
    assert [got[i] for i in pick] == opoa.consensus_batch([groups[i] for i in pick])


def test_32bit_rows_everywhere(monkeypatch):
    """MANDO_POA_DBG=1 forces the 32-bit row loop (4-row LDS ring) for every read: same bytes."""
    monkeypatch.setenv("MANDO_POA_DBG", "1")
    _check(poa_cases.noisy_groups(24, (300, 3500), (3, 20), seed=91)[1])


def test_dense_branching_graphs():
    """Very noisy reads: many rows with 3-5+ predecessors and predecessors several rows back
    (the 16-bit loop's multi-predecessor rows, its 8-row ring and the generic row)."""
    _, g = synth.read_groups(16, (400, 1500), (20, 40), seed=17, model=dict(sub=0.06, ins=0.05, dele=0.05))
    _check(g)
