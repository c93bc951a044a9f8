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
