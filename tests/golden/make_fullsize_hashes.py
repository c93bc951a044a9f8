#!/usr/bin/env python3
"""Generates tests/golden/fullsize_hashes.json: the sha256 of the D module's two output files on bench.py's
FULL-SIZE workloads (config 2: SIRV-like; config 3: 20,000 loci x 50 x 3 kb; config 5: 100 x 200 x 8.5 kb
`-S`; optionally config 4), computed with the CPU restatements in oracle/ (clustering, orientation, POA)
injected into the same driver, on this container's cores.

bench.py compares the GPU run's files after its timed steps against these hashes, so the benchmarked
output is checked as a whole (every locus), not on a sample.  The synthetic data are a pure function of
the workload's parameters and seed (libmando_synth: one RNG stream per locus, independent of threads), so
the GPU box regenerates the same bytes; `records` pins that too.

Usage: python tests/golden/make_fullsize_hashes.py [config2 config3 config5 ...] [--threads 8]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fullsize_hashes.json")


def sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        for blk in iter(lambda: fh.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


def main():
    import bench
    from oracle import cluster as ocl

    ap = argparse.ArgumentParser()
    ap.add_argument("workloads", nargs="*", default=["config2", "config3", "config5"])
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--data-dir", default="/tmp")
    ap.add_argument("--keep", action="store_true", help="keep the generated data")
    a = ap.parse_args()
    out = json.load(open(DST)) if os.path.exists(DST) else {}
    for name in a.workloads:
        wl = bench.WORKLOADS[name]
        d = os.path.join(a.data_dir, f"mando_fullsize_{name}")
        records = bench.gen_data(d, wl, wl["loci"], a.threads)
        of, cf, pool = bench.cpu_fns(a.threads)
        t0 = time.perf_counter()
        try:
            st = bench.run_define(d, a.threads, 0, orient_fn=of, consensus_fn=cf, cluster_fn=ocl.cluster_loci)
        finally:
            pool.shutdown()
        wall = time.perf_counter() - t0
        fa, r2 = os.path.join(d, "Isoform_Consensi.fasta"), os.path.join(d, "reads2isoforms.txt")
        out[f"{name}:{wl['loci']}"] = {
            "records": records, "loci": st["loci"], "isoforms": st["isoforms"], "poa_groups": st["poa_groups"],
            "poa_reads": st["poa_reads"], "isoform_consensi_sha256": sha(fa), "reads2isoforms_sha256": sha(r2),
            "fasta_bytes": os.path.getsize(fa), "r2i_bytes": os.path.getsize(r2),
            "generated_by": f"oracle/ restatements (cluster_ref.cpp, orient_ref.c, poa_ref.c) through "
                            f"mandalorion_amd.define on {a.threads} host threads, {wall:.0f} s"}
        print(name, json.dumps(out[f"{name}:{wl['loci']}"]), flush=True)
        json.dump(out, open(DST, "w"), indent=1, sort_keys=True)
        if not a.keep:
            shutil.rmtree(d, ignore_errors=True)
    print("wrote", DST)


if __name__ == "__main__":
    main()
