# Round-end bench lines of the other workloads (configs 2, 3 and 5), no CPU baseline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08z}
mkdir -p $D
for wl in config2 config3 config5; do
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --workload $wl --steps 5 --warmup 2 > $D/bench_$wl.json 2> $D/bench_$wl.err || { echo "$wl failed"; tail -5 $D/bench_$wl.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$wl.json')); c=d['config']; print('$wl', round(d['value']), round(d['ms_per_step'],1), c['steps_s'], c['steps_poa_kernel_ms'], c.get('full_output_equals_oracle'), c.get('clustering_equals_reference'))"
done
