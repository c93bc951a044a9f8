"""Which hardware queue and stream each kernel of a rocprofv3 kernel trace ran on, with its interval (ms
after the first kernel of the last `--last-ms` window).  Dev helper for the HW-queue sharing question.
usage: python tools/kt_queues.py kernel_trace.csv [--last-ms 3000]"""
import csv
import sys


def main():
    path = sys.argv[1]
    last = float(sys.argv[sys.argv.index("--last-ms") + 1]) if "--last-ms" in sys.argv else 3000.0
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:40],
                     r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
    rows.sort()
    tend = max(x[1] for x in rows)
    rows = [x for x in rows if x[0] >= tend - last * 1e6]
    t0 = rows[0][0]
    # collapse runs of the same kernel on the same queue
    out = []
    for s, e, n, q, st in rows:
        if out and out[-1][2] == n and out[-1][3] == q and out[-1][4] == st and s - out[-1][1] < 2e6:
            out[-1][1] = max(out[-1][1], e)
            out[-1][5] += 1
        else:
            out.append([s, e, n, q, st, 1])
    for s, e, n, q, st, c in out:
        print(f"{(s - t0) / 1e6:9.1f} {(e - t0) / 1e6:9.1f} {(e - s) / 1e6:8.1f}  q{q:>3} s{st:>3}  x{c:<5d} {n}")


if __name__ == "__main__":
    main()
