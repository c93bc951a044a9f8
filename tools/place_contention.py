"""Concurrent placement of an N-rank plan's real output blocks, no GPU work.

tools/rank_rehearsal.py with PLACE_DUMP=<dir> saves, for every rank of an N-rank plan, the blocks it
places into reads2isoforms.txt and Isoform_Consensi.fasta (define._place's arguments: the rank's
formatted bytes, per-root source offsets, its roots, their sizes and the all-rank size table).  This
tool places them the way N rank processes on one node do: N processes, each with `threads` host
threads, a barrier, every rank's reads2isoforms.txt blocks at once, a barrier, every rank's FASTA blocks
at once (the driver's order: reads2isoforms during the POA, the FASTA after it).  For comparison each
rank's blocks are also placed alone, one rank after another.  Rounds alternate concurrent / alone, the
first of each untimed (files created, page cache warm, as in a later bench step).

usage: python tools/place_contention.py <dump dir> <out dir> [threads=2] [rounds=3]
prints one JSON line: per file, the max over ranks of the concurrent placement and the sum / max of
the ranks placed alone.
       python tools/place_contention.py --ranges <out dir> <ranks> <bytes> [threads=2] [rounds=3]
the same for a layout where each rank's blocks are one contiguous range (bytes split evenly).
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FILES = ("reads2isoforms.txt", "Isoform_Consensi.fasta")


def _load(dump: str, rank: int, f: str):
    z = np.load(os.path.join(dump, f"r{rank}_{f}.npz"))
    return {k: z[k] for k in ("buf", "src", "roots", "sizes", "g_sizes")}


def _place(out: str, f: str, b: dict, threads: int) -> float:
    """define._place's work for one rank and file, timed."""
    from mandalorion_amd import _lib

    goff = np.zeros(len(b["g_sizes"]) + 1, np.int64)
    np.cumsum(b["g_sizes"], out=goff[1:])
    t = time.perf_counter()
    fd = os.open(os.path.join(out, f), os.O_RDWR | os.O_CREAT, 0o644)
    try:
        os.ftruncate(fd, int(goff[-1]))
        _lib.write_blocks(fd, b["buf"], b["src"], goff[b["roots"]], b["sizes"], threads=threads)
    finally:
        os.close(fd)
    return time.perf_counter() - t


def _rank(rank, dump, out, threads, rounds, bar, q):
    blocks = {f: _load(dump, rank, f) for f in FILES}
    for _ in range(rounds):
        ts = {}
        for f in FILES:
            bar.wait()
            ts[f] = _place(out, f, blocks[f], threads)
        q.put((rank, ts))


def _range_rank(rank, n, total, out, threads, bar, q):
    part = total // n
    b = {"buf": np.full(part, 65 + rank, np.uint8), "src": np.zeros(1, np.int64), "roots": np.array([rank]),
         "sizes": np.array([part], np.int64), "g_sizes": np.full(n, part, np.int64)}
    bar.wait()
    q.put((rank, {"ranges": _place(out, "ranges.bin", b, threads)}))


def main_ranges():
    out, n, total = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    threads = int(sys.argv[5]) if len(sys.argv) > 5 else 2
    rounds = int(sys.argv[6]) if len(sys.argv) > 6 else 3
    os.makedirs(out, exist_ok=True)
    ctx = mp.get_context("spawn")
    ts = []
    for rd in range(rounds + 1):
        q, bar = ctx.Queue(), ctx.Barrier(n)
        ps = [ctx.Process(target=_range_rank, args=(r, n, total, out, threads, bar, q)) for r in range(n)]
        for p in ps:
            p.start()
        got = [q.get(timeout=600) for _ in range(n)]
        for p in ps:
            p.join(60)
            assert p.exitcode == 0
        if rd:
            ts.append(round(max(t["ranges"] for _, t in got), 4))
    print(json.dumps({"ranks": n, "threads_per_rank": threads, "bytes": total, "layout": "contiguous range per rank",
                      "concurrent_s": ts, "concurrent_median_s": float(np.median(ts))}), flush=True)


def main():
    if sys.argv[1] == "--ranges":
        return main_ranges()
    dump, out = sys.argv[1], sys.argv[2]
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    n = 1 + max(int(x[1:].split("_", 1)[0]) for x in os.listdir(dump) if x.startswith("r") and x.endswith(".npz"))
    os.makedirs(out, exist_ok=True)
    ctx = mp.get_context("spawn")
    res = {"ranks": n, "threads_per_rank": threads, "rounds": rounds, "concurrent_s": {f: [] for f in FILES},
           "alone_sum_s": {f: [] for f in FILES}, "alone_max_s": {f: [] for f in FILES},
           "bytes": {f: int(_load(dump, 0, f)["g_sizes"].sum()) for f in FILES}}
    for rd in range(rounds + 1):
        # concurrent: N processes, barrier per file
        q, bar = ctx.Queue(), ctx.Barrier(n)
        ps = [ctx.Process(target=_rank, args=(r, dump, out, threads, 1, bar, q)) for r in range(n)]
        for p in ps:
            p.start()
        got = [q.get(timeout=600) for _ in range(n)]
        for p in ps:
            p.join(60)
            assert p.exitcode == 0
        # alone: one rank at a time, in this process
        alone = {f: [_place(out, f, _load(dump, r, f), threads) for r in range(n)] for f in FILES}
        if rd == 0:
            continue
        for f in FILES:
            res["concurrent_s"][f].append(round(max(ts[f] for _, ts in got), 4))
            res["alone_sum_s"][f].append(round(sum(alone[f]), 4))
            res["alone_max_s"][f].append(round(max(alone[f]), 4))
    res["concurrent_median_s"] = {f: float(np.median(v)) for f, v in res["concurrent_s"].items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
