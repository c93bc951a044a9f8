"""Dev tool: the POA groups a workload hands the kernel, by band (CPU only; the oracle's clustering and
orientation, the driver's assembly): group depth, mean read length, the band 2w + 1 of abPOA's adaptive
band at that length (w = 10 + 0.01 L), which launch kind takes them (narrow <= 116 < wide) and their share
of the DP cells (estimated as (n - 1) x L x 1.15 x min(band, L)).
usage: python tools/group_census.py [workload=config4] [loci=3000]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from mandalorion_amd import define  # noqa: E402
from oracle import cluster as ocl, orient as oref  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "config4"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
    d = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"mando_census_{wl}_{n}")
    os.makedirs(d, exist_ok=True)
    recs = bench.gen_data(d, bench.WORKLOADS[wl], n, 8)
    G = []

    def cons_fn(seqs, seq_off, grp_off, seeding):
        lens = np.diff(seq_off)
        cons, off = [], [0]
        for g in range(len(grp_off) - 1):
            ln = lens[grp_off[g]:grp_off[g + 1]]
            G.append((len(ln), float(ln.mean())))
            a, b = seq_off[grp_off[g]], seq_off[grp_off[g] + 1]
            cons.append(np.frombuffer(bytes(seqs[a:b]), dtype=np.uint8))
            off.append(off[-1] + b - a)
        return (np.concatenate(cons) if cons else np.zeros(0, np.uint8)), np.array(off, dtype=np.int64)

    t = time.time()
    define.define_isoforms(d, threads=6, device=0, orient_fn=oref.orient_packed, consensus_fn=cons_fn,
                           cluster_fn=ocl.cluster_loci)
    g = np.array(G)
    depth, mean = g[:, 0], g[:, 1]
    band = 2 * (10 + (0.01 * mean).astype(int)) + 1
    cells = (depth - 1) * mean * 1.15 * np.minimum(band, mean)
    print(f"{wl}: {n} loci, {recs} records, {len(g)} POA groups ({time.time() - t:.0f} s)")
    print("depth percentiles 5/25/50/75/95:", np.percentile(depth, [5, 25, 50, 75, 95]).tolist())
    print("mean read length percentiles 5/25/50/75/95/99:", np.round(np.percentile(mean, [5, 25, 50, 75, 95, 99])).tolist())
    print("band percentiles 5/25/50/75/95/99:", np.percentile(band, [5, 25, 50, 75, 95, 99]).tolist())
    wide = band > 116
    print(f"wide launch: {int(wide.sum())} groups ({wide.mean():.4f}), {cells[wide].sum() / cells.sum():.4f} of the cells")
    for lo, hi in [(0, 65), (65, 81), (81, 97), (97, 105), (105, 113), (113, 117), (117, 129), (129, 10 ** 6)]:
        m = (band > lo) & (band <= hi)
        print(f"  band ({lo}, {hi}]: {int(m.sum())} groups, {cells[m].sum() / cells.sum():.3f} of the cells")


if __name__ == "__main__":
    main()
