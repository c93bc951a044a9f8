"""Turns two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, MI355X_MICROARCH.md "HBM")
of `bench.py --steps 1 --warmup 0` into profiles/pmc_latest.json, which bench.py reads for
roofline.traffic.  The pass runs ONE step, so the POA dispatches' sums are the HBM bytes per step.
gfx950 correction: FETCH_SIZE counts half the bytes of wide coalesced reads, so it is doubled;
WRITE_SIZE is taken as is.  Counter values are in KiB (rocprofv3 derived metrics).  The file records the
chunk plan and the POA dispatch count of that step: bench.py uses the traffic only when its own step has
the same plan, chunk count and dispatch count (and the same POA sources).
usage: python tools/pmc_traffic.py fetch.csv write.csv WORKLOAD CHUNKS [out.json]"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collections import defaultdict


def per_dispatch(path, counter, kernel="poa_kernel"):
    vals = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r.get("Dispatch_Id", "0")] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    import bench

    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    if len(fetch) != len(write):
        raise SystemExit(f"the passes saw {len(fetch)} and {len(write)} POA dispatches")
    f = sum(fetch) * 1024.0
    w = sum(write) * 1024.0
    out = {"workload": sys.argv[3], "chunks": int(sys.argv[4]), "plan": bench.plan_signature(),
           "poa_dispatches_per_step": len(fetch), "fetch_size_bytes_raw_per_step": f,
           "write_size_bytes_per_step": w, "hbm_bytes_per_step": 2.0 * f + w, "hbm_bytes_per_step_raw": f + w,
           # the guide calibrates the x2 only for 16-B-per-lane streaming reads; the kernel's reads are
           # mixed (int4 window / descriptor loads, dword and short loads), so the raw sum is the lower
           # and the doubled fetch the upper estimate
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE x1; KiB -> bytes; raw = x1",
           # provenance: bench.py uses the traffic only when the POA sources it runs hash the same
           "commit": os.environ.get("MANDO_COMMIT", "unknown"), "poa_sources_sha256": bench.poa_sources_sha()}
    dst = sys.argv[5] if len(sys.argv) > 5 else "profiles/pmc_latest.json"
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
