"""Summarises a MANDO_WG_TRACE file (one line per workgroup of each one-group POA launch: batch, kind,
block, group, t0, t1 (100 MHz ticks), HW_ID, XCC_ID, reads) per launch: duration, the slowest workgroup,
its placement, and how many other wide workgroups shared its SIMD / CU while it ran.
usage: python tools/wg_trace.py trace.txt"""
import sys
from collections import defaultdict


def place(hw, xcc):
    # gfx9 HW_ID: wave [3:0], simd [5:4], pipe [7:6], cu [11:8], sh [12], se [15:13]
    return (xcc & 15, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15, (hw >> 4) & 3)


def main():
    rows = defaultdict(list)
    for line in open(sys.argv[1]):
        b, k, blk, g, t0, t1, hw, xcc, nr = map(int, line.split())
        if t1 > 0:
            rows[(b, k)].append((t0, t1, place(hw, xcc), g, nr, blk))
    for (b, k), L in sorted(rows.items()):
        start = min(x[0] for x in L)
        end = max(x[1] for x in L)
        slow = max(L, key=lambda x: x[1])
        t0, t1, pl, g, nr, blk = slow
        same_simd = sum(1 for x in L if x is not slow and x[2] == pl and x[0] < t1 and x[1] > t0)
        same_cu = sum(1 for x in L if x is not slow and x[2][:4] == pl[:4] and x[0] < t1 and x[1] > t0)
        durs = sorted((x[1] - x[0]) / 1e5 for x in L)
        print(f"batch {b} kind {k}: {len(L)} wgs, launch {(end - start) / 1e5:7.1f} ms; slowest wg {blk} group {g} "
              f"({nr} reads) {(t1 - t0) / 1e5:7.1f} ms (start +{(t0 - start) / 1e5:.1f} ms) at xcc/se/sh/cu/simd {pl}; "
              f"other {'wide' if k == 1 else 'same-kind'} wgs on its SIMD {same_simd}, on its CU {same_cu}; "
              f"median wg {durs[len(durs) // 2]:.1f} ms, 2nd slowest {durs[-2] if len(durs) > 1 else 0:.1f} ms")


if __name__ == "__main__":
    main()
