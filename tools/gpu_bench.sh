# GPU box: default bench line, then a rocprofv3 kernel-trace summary of one e2e step.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-b}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python bench.py ${BARGS:-} > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
if [ -z "$NOPROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BARGS:-} > $D/prof.out 2>&1 || { echo "prof failed"; tail -5 $D/prof.out; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
fi
