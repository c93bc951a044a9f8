"""Concurrent page-cache reads of an N-rank plan's locus files, no GPU work.

The rank rehearsal (tools/rank_rehearsal.py) runs the ranks of a plan one after another, so each rank
reads its share of the locus text from the page cache alone.  In an N-GPU run the N ranks read at once,
from one page cache.  This tool reads the real shares of the plan the D driver builds (define._lpt_owner
over define._size_costs of the sorted roots) the way the ranks do: N processes, `threads` reader threads
each, a barrier, every rank reading its own files into its own buffer.  For comparison one rank's share
is also read alone.  Rounds alternate (concurrent, alone); the first round is untimed (page cache warm,
as in a later bench step).  Before the rounds, the page-cache residency of every file is taken with
mincore (bench.page_cache_resident).

usage: python tools/read_contention.py <data dir holding tmp_SS> <ranks> [threads=2] [rounds=3]
prints one JSON line.
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def read_files(files: list, sizes: np.ndarray, threads: int) -> float:
    off = np.concatenate([[0], np.cumsum(sizes)])
    buf = np.empty(max(int(off[-1]), 1), np.uint8)
    buf[::4096] = 0  # pages faulted in before the clock: the driver's pinned buffer is reused across calls
    mv = memoryview(buf)
    nxt = [0]
    lock = threading.Lock()

    def work():
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= len(files):
                return
            fd = os.open(files[i], os.O_RDONLY)
            try:
                os.readv(fd, [mv[off[i]:off[i + 1]]])
            finally:
                os.close(fd)

    t = time.perf_counter()
    th = [threading.Thread(target=work) for _ in range(threads)]
    [x.start() for x in th]
    [x.join() for x in th]
    return time.perf_counter() - t


def rank_main(r, files, sizes, threads, rounds, bar, q):
    out = []
    for k in range(rounds):
        bar.wait()
        dt = read_files(files, sizes, threads)
        bar.wait()
        out.append(dt)
    q.put((r, out))


def main():
    import bench
    from mandalorion_amd import define

    data, world = sys.argv[1], int(sys.argv[2])
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    tmp = os.path.join(data, "tmp_SS")
    size_arr: list = []
    roots = define._roots(tmp, size_array=size_arr)
    sizes = size_arr[0]
    owner = define._lpt_owner(define._size_costs(sizes), world)
    files = [os.path.join(tmp, r + ".psl") for r in roots]
    shares = [np.flatnonzero(owner == r) for r in range(world)]
    resident = bench.page_cache_resident(files)
    ctx = mp.get_context("fork")
    res = {"ranks": world, "threads_per_rank": threads, "files": len(files), "bytes": int(sizes.sum()),
           "share_bytes": [int(sizes[s].sum()) for s in shares], "page_cache_resident": resident,
           "concurrent_s": [], "alone_rank0_s": []}
    for k in range(rounds):
        bar = ctx.Barrier(world)
        q = ctx.Queue()
        ps = [ctx.Process(target=rank_main, args=(r, [files[i] for i in shares[r]], sizes[shares[r]], threads, 1,
                                                   bar, q)) for r in range(world)]
        [p.start() for p in ps]
        got = dict(q.get() for _ in ps)
        [p.join() for p in ps]
        conc = max(v[0] for v in got.values())
        alone = read_files([files[i] for i in shares[0]], sizes[shares[0]], threads)
        if k:
            res["concurrent_s"].append(round(conc, 4))
            res["alone_rank0_s"].append(round(alone, 4))
        print(f"round {k}: concurrent max {conc:.3f} s, rank 0 alone {alone:.3f} s", file=sys.stderr, flush=True)
    if res["concurrent_s"]:
        c = float(np.median(res["concurrent_s"]))
        res["concurrent_median_s"] = c
        res["aggregate_GBps"] = round(res["bytes"] / c / 1e9, 2)
        res["alone_rank0_GBps"] = round(res["share_bytes"][0] / float(np.median(res["alone_rank0_s"])) / 1e9, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
