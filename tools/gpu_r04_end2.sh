# GPU box, round end after the chunk-plan change: every GPU test, smoke, and the default bench line
# (config 4, N=1, with the CPU baseline) as the driver runs it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04e2}_tests bash tools/gpu_r04_tests.sh || exit 1
D=gpurun_out/${TAG:-r04e2}
mkdir -p $D
timeout -k 10 900 python3 bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench failed"; tail -5 $D/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_default.json')); c=d['config']; print(round(d['value']), round(d['ms_per_step'], 1), c['steps_s'], c.get('chunks'), c.get('full_output_equals_oracle'), d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline'])"
