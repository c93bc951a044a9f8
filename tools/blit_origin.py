"""Dev tool: where the runtime's shader copies (`__amd_rocclr_copyBuffer` / fill kernels) of a D-module run
come from, and what occupies the GPU between POA launches.

Input: a rocprofv3 output directory of `--kernel-trace --memory-copy-trace --hip-runtime-trace
--output-format csv` (no PMC).  For every blit dispatch it joins the kernel record with the HIP API call
of the same correlation id, prints the API calls around it on the same host thread, and sums the blits
per API function; then lists the POA launches (narrow / wide kernels) with the gaps between consecutive
launch pairs and the kernels and copies that ran in each gap.

usage: python tools/blit_origin.py <rocprofv3 output dir> [max blits listed=40]
"""
from __future__ import annotations

import collections
import csv
import glob
import os
import sys


def load(d: str, pat: str) -> list:
    fs = glob.glob(os.path.join(d, "**", f"*{pat}"), recursive=True)
    rows = []
    for f in fs:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def col(row: dict, *names):
    for n in names:
        for k in row:
            if k.lower() == n.lower():
                return row[k]
    return None


def main():
    d = sys.argv[1]
    lim = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    kt = load(d, "kernel_trace.csv")
    api = load(d, "hip_api_trace.csv")
    mc = load(d, "memory_copy_trace.csv")
    print(f"{len(kt)} kernel dispatches, {len(api)} HIP API calls, {len(mc)} DMA copies")
    for r in kt:
        r["_s"], r["_e"] = int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp"))
        r["_n"] = col(r, "Kernel_Name") or "?"
        r["_c"] = col(r, "Correlation_Id")
        r["_q"] = col(r, "Queue_Id") or col(r, "Stream_Id") or "?"
    by_corr = {col(a, "Correlation_Id"): a for a in api}
    by_thread = collections.defaultdict(list)
    for a in api:
        a["_s"] = int(col(a, "Start_Timestamp"))
        by_thread[col(a, "Thread_Id")].append(a)
    for t in by_thread.values():
        t.sort(key=lambda a: a["_s"])
    pos = {id(a): i for t in by_thread.values() for i, a in enumerate(t)}
    t0 = min(r["_s"] for r in kt) if kt else 0
    blits = [r for r in kt if "rocclr" in r["_n"]]
    print(f"\n{len(blits)} runtime blit dispatches")
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for i, b in enumerate(sorted(blits, key=lambda r: r["_s"])):
        a = by_corr.get(b["_c"])
        fn = col(a, "Function") if a else "?"
        dur = (b["_e"] - b["_s"]) / 1e6
        key = (b["_n"].split("(")[0], fn)
        agg[key][0] += 1
        agg[key][1] += dur
        agg[key][2] = max(agg[key][2], dur)
        if i < lim:
            ctx = ""
            if a is not None:
                th = by_thread[col(a, "Thread_Id")]
                j = pos[id(a)]
                ctx = " | before: " + ", ".join(col(x, "Function") for x in th[max(0, j - 4):j]) + \
                      " | after: " + ", ".join(col(x, "Function") for x in th[j + 1:j + 3])
            grid = col(b, "Grid_Size_X") or col(b, "Grid_Size") or "?"
            print(f"  t={(b['_s'] - t0) / 1e9:8.3f}s dur {dur:8.3f} ms q {b['_q']} grid {grid} "
                  f"{b['_n'].split('(')[0]} <- {fn} (thread {col(a, 'Thread_Id') if a else '?'}){ctx}")
    print("\nblits by (kernel, API function): count, total ms, max ms")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k[0]:40s} {k[1]:28s} {v[0]:5d} {v[1]:10.1f} {v[2]:8.1f}")
    # POA launch pairs and what runs between them
    poa = sorted([r for r in kt if r["_n"].startswith("void mando::poa_kernel") or "poa_kernel" in r["_n"]],
                 key=lambda r: r["_s"])
    if not poa:
        return
    # group launches that overlap into batches
    batches = []
    for r in poa:
        if batches and r["_s"] < batches[-1][1]:
            batches[-1][1] = max(batches[-1][1], r["_e"])
            batches[-1][2].append(r)
        else:
            batches.append([r["_s"], r["_e"], [r]])
    print(f"\n{len(batches)} POA batches (overlapping launches merged)")
    others = sorted([r for r in kt if "poa_kernel" not in r["_n"]], key=lambda r: r["_s"])
    for c in mc:
        c["_s"], c["_e"] = int(col(c, "Start_Timestamp")), int(col(c, "End_Timestamp"))
    gap_tot = 0.0
    for i, (s, e, rs) in enumerate(batches):
        line = f"  batch {i:2d}: {(s - t0) / 1e9:8.3f} -> {(e - t0) / 1e9:8.3f} s ({(e - s) / 1e6:8.1f} ms, {len(rs)} launches)"
        if i + 1 < len(batches):
            g0, g1 = e, batches[i + 1][0]
            gap_tot += (g1 - g0) / 1e6
            inside = collections.Counter()
            for r in others:
                if r["_e"] > g0 and r["_s"] < g1:
                    inside[r["_n"].split("(")[0][-40:]] += 1
            dma = sum(1 for c in mc if c["_e"] > g0 and c["_s"] < g1)
            line += f"; gap {(g1 - g0) / 1e6:7.1f} ms: {dict(inside)} + {dma} DMA copies"
        print(line)
    print(f"  sum of gaps between POA batches: {gap_tot:.1f} ms")


if __name__ == "__main__":
    main()
