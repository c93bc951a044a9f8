# GPU box: the PMC HBM passes (FETCH_SIZE, WRITE_SIZE; separate runs) of one config-3 step at the current
# sources -> gpurun_out/$TAG/pmc_latest.json (copy to profiles/pmc_latest.json), then a bench line reading it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-pmc}
mkdir -p $D
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $D/pmcf -o f --output-format csv -- $B --steps 1 --warmup 0 > $D/pmcf.out 2>&1 || { echo "pmcf failed"; tail -5 $D/pmcf.out; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $D/pmcw -o w --output-format csv -- $B --steps 1 --warmup 0 > $D/pmcw.out 2>&1 || { echo "pmcw failed"; tail -5 $D/pmcw.out; exit 1; }
F=$(find $D/pmcf -name "*counter_collection.csv" | head -1); W=$(find $D/pmcw -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py $F $W config3:20000 $D/pmc_latest.json || exit 1
timeout -k 10 300 $B --pmc-json $D/pmc_latest.json > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -5 $D/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench.json')); print(d['value'], d['roofline'])"
