"""Turns two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, MI355X_MICROARCH.md "HBM")
of `bench.py --steps 1 --warmup 0` into profiles/pmc_latest.json, which bench.py reads for
roofline.traffic.  gfx950 correction: FETCH_SIZE counts half the bytes of wide coalesced reads, so it
is doubled; WRITE_SIZE is taken as is.  Counter values are in KiB (rocprofv3 derived metrics).
usage: python tools/pmc_traffic.py fetch.csv write.csv WORKLOAD [out.json]"""
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
    f = sum(fetch) / max(len(fetch), 1) * 1024.0
    w = sum(write) / max(len(write), 1) * 1024.0
    out = {"workload": sys.argv[3], "fetch_size_bytes_raw": f, "write_size_bytes": w,
           "hbm_bytes_per_launch": 2.0 * f + w, "hbm_bytes_per_launch_raw": f + w,
           "dispatches": [len(fetch), len(write)],
           # the guide calibrates the x2 only for 16-B-per-lane streaming reads; the kernel's reads are
           # mixed (int4 window / descriptor loads, dword and short loads), so the raw sum is the lower
           # and the doubled fetch the upper estimate
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE x1; KiB -> bytes; raw = x1",
           # provenance: bench.py uses the traffic only when the POA sources it runs hash the same
           "commit": os.environ.get("MANDO_COMMIT", "unknown"), "poa_sources_sha256": bench.poa_sources_sha()}
    dst = sys.argv[4] if len(sys.argv) > 4 else "profiles/pmc_latest.json"
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
