"""Regenerate tests/golden/rng_vectors.json from numpy's legacy RandomState (the reference's RNG).

Each case replays `np.random.seed(seed)` then `np.random.choice(np.arange(n), min(n,k), replace=False)`
for each (n, k) in order — the call pattern of utils/SpliceDefineConsensus.py:505/:818/:884.
"""
import json
import os

import numpy as np

CASES = [
    (0, [(1, 1), (2, 2), (5, 5), (40, 40), (600, 500), (150, 100)]),
    (7, [(6, 6), (6, 6), (6, 6), (6, 6)]),
    (20250117, [(17, 17), (333, 100), (1000, 500), (3, 3)]),
    (4294967295, [(64, 64), (65, 65), (129, 100)]),
]


def main():
    out = []
    for seed, draws in CASES:
        np.random.seed(seed)
        vals = [np.random.choice(np.arange(0, n), min(n, k), replace=False).tolist() for n, k in draws]
        out.append({"seed": seed, "draws": draws, "out": vals})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rng_vectors.json")
    json.dump({"generator": "numpy legacy RandomState " + np.__version__, "cases": out}, open(path, "w"))


if __name__ == "__main__":
    main()
