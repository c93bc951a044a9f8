# Round profile on the GPU box: PMC HBM passes (FETCH_SIZE, WRITE_SIZE; separate runs) over one step of
# the default bench (WL, default config4: the whole D module), the bench line reading the PMC traffic just
# measured, a rocprofv3 kernel-trace summary of the same command, and one SQ pass (issue / wait cycles)
# of the POA kernel.  usage: TAG=r02e bash tools/profile_round.sh   (outputs under gpurun_out/$TAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-prof}
mkdir -p $D
export TMPDIR=/tmp
WL=${WL:-config4}
KEY=$(python3 -c "import bench; print('$WL:%d' % bench.WORKLOADS['$WL']['loci'])")
B="python3 bench.py --no-cpu-baseline --workload $WL"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $D/pmcf -o f --output-format csv -- $B --steps 1 --warmup 0 > $D/pmcf.out 2>&1 || { echo "pmcf failed"; tail -5 $D/pmcf.out; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $D/pmcw -o w --output-format csv -- $B --steps 1 --warmup 0 > $D/pmcw.out 2>&1 || { echo "pmcw failed"; tail -5 $D/pmcw.out; exit 1; }
F=$(find $D/pmcf -name "*counter_collection.csv" | head -1); W=$(find $D/pmcw -name "*counter_collection.csv" | head -1)
CH=$(python3 -c "import json; print([json.loads(l) for l in open('$D/pmcf.out') if l.startswith('{\"metric')][-1]['config']['chunks'])") || exit 1
python3 tools/pmc_traffic.py $F $W $KEY $CH $D/pmc_latest.json || exit 1
timeout -k 10 600 python3 bench.py --workload $WL --pmc-json $D/pmc_latest.json > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -5 $D/bench.err; exit 1; }
cat $D/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- $B --steps 3 --warmup 1 --pmc-json $D/pmc_latest.json > $D/prof.out 2>&1 || { echo "prof failed"; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -1 | xargs head -6
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $D/pmcsq -o s --output-format csv -- $B --steps 1 --warmup 0 > $D/pmcsq.out 2>&1 || { echo "sq pass failed"; tail -5 $D/pmcsq.out; exit 1; }
python3 tools/pmc_sq.py $(find $D/pmcsq -name "*counter_collection.csv" | head -1) > $D/sq.txt && cat $D/sq.txt
