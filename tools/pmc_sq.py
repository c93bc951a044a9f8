"""Summarises one rocprofv3 SQ counter pass per kernel: waves, wave cycles split into active-issue /
issue-stall / parked (MI355X_MICROARCH.md "rocprofv3 PMC slots": WAIT_ANY + WAIT_INST_ANY +
ACTIVE_INST_ANY ~ WAVE_CYCLES, all in quad-cycles), and instructions per wave by type.
usage: python tools/pmc_sq.py counter_collection.csv"""
import csv
import sys
from collections import defaultdict


def main():
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(sys.argv[1])):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].strip()
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", "0"))
    for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        w = c.get("SQ_WAVES", 0) or 1
        print(f"{k}: dispatches {len(disp[k])}, waves {c.get('SQ_WAVES', 0):.0f}, wave-cycles {4 * wc:.3e} "
              f"(active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.1%}, issue-stall {c.get('SQ_WAIT_INST_ANY', 0) / wc:.1%}, "
              f"parked {c.get('SQ_WAIT_ANY', 0) / wc:.1%}); per wave: VALU {c.get('SQ_INSTS_VALU', 0) / w:.3e}, "
              f"SALU {c.get('SQ_INSTS_SALU', 0) / w:.3e}, LDS {c.get('SQ_INSTS_LDS', 0) / w:.3e}")


if __name__ == "__main__":
    main()
