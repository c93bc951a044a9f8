"""bench.py's own launcher (`--gpus N` without WORLD_SIZE): N rank processes, a rendezvous, the data on
rank 0 and the driver's LPT shard plan.  `--check-launch` stops before any GPU compute, so this runs on
the CPU over the host transport; on a GPU box the same launcher feeds the timed run, which then requires
RCCL on every rank (bench.py main)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, gpus):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--check-launch",
                        "--workload", "config3", "--loci", "64", "--data-dir", str(tmp_path)],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # one JSON line, from rank 0 only
    return json.loads(lines[0])


def test_bench_spawns_two_ranks(tmp_path):
    out = _run(tmp_path, 2)
    assert out["n_gpus"] == 2 and out["world"] == 2
    assert out["backend"] == "host"
    assert [r["rank"] for r in out["ranks"]] == [0, 1]
    assert sum(r["loci"] for r in out["ranks"]) == 64
    assert all(r["loci"] > 0 for r in out["ranks"])
    assert out["records"] == 64 * 50


def test_bench_one_rank_plan(tmp_path):
    out = _run(tmp_path, 1)
    assert out["n_gpus"] == 1 and out["ranks"][0]["loci"] == 64
