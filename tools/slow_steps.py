"""Slow-step forensics from a rocprofv3 kernel trace of bench.py (config 3): per step, each POA launch's
duration and start offset, and the other kernels that overlap it (name, count, busy ms).
usage: python tools/slow_steps.py kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Stream_Id", r.get("Queue_Id", "?"))))
    rows.sort()
    poa = [x for x in rows if "poa_kernel" in x[2]]
    # steps: the first launch of chunk 1 follows a gap; group POA launches into steps by the clustering
    # launches that precede them (a step starts with cluster_parse of its first chunk)
    starts = [x[0] for x in rows if "cluster_parse" in x[2]]
    # two chunks per step: every other cluster_parse begins a step
    step_starts = starts[0::2]
    def step_of(t):
        k = 0
        while k + 1 < len(step_starts) and step_starts[k + 1] <= t:
            k += 1
        return k
    by_step = defaultdict(list)
    for x in poa:
        by_step[step_of(x[0])].append(x)
    for k in sorted(by_step):
        t0 = step_starts[k]
        tot = 0.0
        print(f"step {k}:")
        for (a, b, name, q) in by_step[k]:
            kind = "wide" if "Li256" in name else ("seeded" if "Lb1" in name else "narrow")
            dur = (b - a) / 1e6
            tot += dur
            ov = defaultdict(lambda: [0, 0.0])
            for (c, d, n2, q2) in rows:
                if d <= a or c >= b or (c, d, n2) == (a, b, name):
                    continue
                key = n2.split("(")[0].split("<")[0][-40:]
                ov[key][0] += 1
                ov[key][1] += (min(b, d) - max(a, c)) / 1e6
            others = ", ".join(f"{n} x{c} {ms:.0f}ms" for n, (c, ms) in sorted(ov.items(), key=lambda kv: -kv[1][1])[:5])
            print(f"   {kind:6s} start +{(a - t0) / 1e6:8.1f} ms  dur {dur:8.1f} ms  stream {q}  beside: {others}")
        print(f"   POA total {tot:.1f} ms")


if __name__ == "__main__":
    main()
