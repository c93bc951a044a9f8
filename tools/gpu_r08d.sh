# Instruction-cache counters of the POA, clustering and orientation kernels (one config-3 step, PMC:
# dispatches serialised), for the slow-launch question.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08d}
mkdir -p $D
timeout -k 10 300 python3 bench.py --workload config3 --no-cpu-baseline --steps 1 --warmup 0 > $D/warm.json 2> $D/warm.err || { echo "warm failed"; tail -5 $D/warm.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $D/sqc -o sqc --output-format csv -- python3 bench.py --workload config3 --no-cpu-baseline --steps 1 --warmup 0 > $D/sqc.out 2>&1 || { echo "sqc pass failed"; tail -5 $D/sqc.out; exit 1; }
python3 - $D <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
f = glob.glob(d + "/sqc/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0][-60:]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVE_CYCLES":
        n[k] += 1
out = open(d + "/sqc_summary.txt", "w")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    h, m = v.get("SQC_ICACHE_HITS", 0), v.get("SQC_ICACHE_MISSES", 0)
    line = (f"{k:60s} dispatches {n[k]:3d} icache hits {h:.3e} misses {m:.3e} (miss rate {m / max(h + m, 1):.4f}) "
            f"dup {v.get('SQC_ICACHE_MISSES_DUPLICATE', 0):.3e} ifetch {v.get('SQ_IFETCH', 0):.3e} "
            f"wait_inst_any/wave_cycles {v.get('SQ_WAIT_INST_ANY', 0) / max(v.get('SQ_WAVE_CYCLES', 1), 1):.4f}")
    print(line)
    out.write(line + "\n")
PY
