"""The POA oracle (oracle/poa_ref.c, abPOA restatement, parity UNPINNED vs real abPOA) behaves like a
POA consensus caller: recovers templates from noisy R2C2-like reads, is deterministic, and handles the
edge cases the reference can produce.  CPU only."""
import numpy as np

from oracle import poa as opoa
from tests import poa_cases


def test_recovers_templates_from_noisy_reads():
    templates, groups = poa_cases.noisy_groups(12, (300, 900), (8, 20), seed=5)
    cons = opoa.consensus_batch(groups)
    exact = sum(c == t for c, t in zip(cons, templates))
    assert exact >= 10, exact


def test_deterministic_and_batch_independent():
    _, groups = poa_cases.noisy_groups(6, 400, 10, seed=9)
    a = opoa.consensus_batch(groups)
    b = [opoa.consensus_batch([g])[0] for g in groups]
    assert a == b


def test_edge_cases():
    groups = poa_cases.edge_groups()
    cons, cells = opoa.consensus_batch(groups, return_cells=True)
    assert cons[0] == groups[0][0]                 # single read is its own consensus
    assert cons[1] == groups[1][0] and cons[2] == groups[2][0]
    assert cons[11] == "" and cells[11] == 0       # empty group
    assert cons[8] in ("A", "C")
    assert all(set(c) <= set("ACGTN") for c in cons)
    assert cells[0] == 0 and cells[1] > 0


def test_cells_follow_band_model():
    # chain of L nodes aligned by an identical read: rows L+1 (source included), width <= 2w+1+1
    t = "".join(np.random.default_rng(1).choice(list("ACGT"), 1000))
    _, cells = opoa.consensus_batch([[t, t]], return_cells=True)
    w = 10 + int(0.01 * 1000)
    assert (len(t) + 1) * (w + 1) < cells[0] <= (len(t) + 1) * (2 * w + 2)


# ---- -S (seeded window partition) restatement -------------------------------------------------
def test_seeded_partition_properties():
    from mandalorion_amd import synth

    p = opoa.Params.defaults()
    _, groups = synth.read_groups(3, (8000, 9000), (3, 3), seed=17)
    for g in groups:
        t, q = g[0], g[1]
        par = opoa.seed_partition(t, q)
        assert len(par) >= 10
        T = Q = 0
        for a, b in par:  # kept anchors are >= min_w apart and >= min_w from both ends
            assert a - T >= p.min_w and b - Q >= p.min_w
            assert len(t) - (a + p.k) >= p.min_w and len(q) - (b + p.k) >= p.min_w
            assert t[a:a + p.k] == q[b:b + p.k]  # equal hash + strand => equal k-mer
            T, Q = a + p.k, b + p.k


def test_seeded_recovers_templates_with_fewer_cells():
    from mandalorion_amd import synth

    templates, groups = synth.read_groups(4, (8000, 9000), (8, 14), seed=5)
    a, ca = opoa.consensus_batch(groups, return_cells=True, seeding=[1] * 4)
    b, cb = opoa.consensus_batch(groups, return_cells=True)
    assert sum(x == t for x, t in zip(a, templates)) >= 3
    assert all(x < y / 3 for x, y in zip(ca, cb))  # windows: narrow bands instead of one 8 kb band


def test_seeded_short_reads_equal_unseeded():
    """Reads too short for two min_w windows get no anchor: the -S path is then the plain DP."""
    _, groups = poa_cases.noisy_groups(6, (300, 1000), (5, 12), seed=3)
    a, ca = opoa.consensus_batch(groups, return_cells=True, seeding=[1] * 6)
    b, cb = opoa.consensus_batch(groups, return_cells=True)
    assert a == b and list(ca) == list(cb)


def test_seeded_edge_cases():
    groups = poa_cases.edge_groups()
    a = opoa.consensus_batch(groups, seeding=[1] * len(groups))
    b = opoa.consensus_batch(groups)
    assert a == b
    # N runs and a read that shares no k-mer with its predecessor
    rng = np.random.default_rng(4)
    t = "".join(rng.choice(list("ACGT"), 3000))
    u = "".join(rng.choice(list("ACGT"), 3000))
    g = [t, t[:1200] + "N" * 50 + t[1250:], u, t, t]
    c = opoa.consensus_batch([g], seeding=[1])[0]
    assert c == t
