# GPU box: step-to-step spread of the headline lines: config 4 over 10 steps, config 3 over 20.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04s10}
mkdir -p $D
timeout -k 10 900 python3 bench.py --no-cpu-baseline --workload config4 --steps 10 --warmup 1 > $D/bench_config4_10.json 2> $D/bench_config4_10.err || { echo c4 failed; tail -5 $D/bench_config4_10.err; exit 1; }
timeout -k 10 600 python3 bench.py --no-cpu-baseline --workload config3 --steps 20 --warmup 1 > $D/bench_config3_20.json 2> $D/bench_config3_20.err || { echo c3 failed; tail -5 $D/bench_config3_20.err; exit 1; }
for f in $D/bench_config4_10.json $D/bench_config3_20.json; do
  python3 -c "import json, statistics as st; d=json.load(open('$f')); s=d['config']['steps_s']; m=st.median(s); print('$f', round(d['value']), 'median', m, 'max/median', round(max(s)/m, 3), s)"
done
