"""Shared POA test cases (seeded).  Edge cases mirror what the reference path can hand abPOA:
single reads, identical reads, ragged ends, N bases / lowercase (abPOA maps them like uppercase / N),
empty reads, unrelated reads (band edges, garbage cells), long indels (far predecessors, wide bands)."""
import numpy as np

from mandalorion_amd import synth


def _rs(rng, n):
    return synth.BASES[rng.integers(0, 4, size=n)].tobytes().decode()


def edge_groups(seed=11):
    rng = np.random.default_rng(seed)
    t = _rs(rng, 300)
    g = []
    g.append([t])                                           # single read
    g.append([t, t])                                        # identical pair
    g.append([t, t, t, t, t])                               # identical, deeper
    g.append([t[:200], t[50:], t[20:280], t])               # ragged ends
    g.append([t, t[:120] + "N" * 5 + t[125:], t.lower()])   # N and lowercase
    g.append([t, "", t[::-1], ""])                          # empty reads are skipped
    g.append([_rs(rng, 250), _rs(rng, 260), _rs(rng, 240)]) # unrelated reads
    g.append([t, t[:100] + _rs(rng, 90) + t[100:], t, t[:150] + t[230:], t])  # long ins / del
    g.append(["A", "C", "A"])                               # length-1 reads
    g.append(["ACGT" * 40, "ACGT" * 38 + "AC", "ACGTACGA" * 20])  # repeats
    g.append([t[:30], t[:60], t[:90]])                      # prefixes
    g.append([])                                            # empty group
    return g


def noisy_groups(n, length, depth, seed):
    return synth.read_groups(n, length, depth, seed=seed)
