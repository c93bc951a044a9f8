# GPU box: why is the second call of a process slow in the rank rehearsal? (WS log: slots, budgets, hipMalloc times)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04i}
mkdir -p $D
timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload config3 --steps 1 --warmup 0 > $D/b.json 2> $D/b.err || exit 1
MANDO_WS_LOG=1 timeout -k 10 600 python3 tools/rank_rehearsal.py /tmp/mando_bench_config3_20000 4 16 > $D/reh.json 2> $D/reh.err || { tail -5 $D/reh.err; exit 1; }
cat $D/reh.json | cut -c1-400
grep -E "mando ws|slot workspace" $D/reh.err | cut -c1-200 | head -60
