# GPU box, round 4: two-wave wide groups -- parity tests first (bounded), then a config-5 A/B (1 vs 2 waves).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04b}
mkdir -p $D
timeout -k 10 60 ./tools/ubench_xwave > $D/ubench_xwave.txt 2>&1 && cat $D/ubench_xwave.txt || exit 1
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 200 --timeout-method thread -k "wide_launch_waves or two_waves_deep or grid_modes or wide_band" > $D/pytest_w2.log 2>&1
rc=$?; grep -E "passed|failed" $D/pytest_w2.log | tail -2 | cut -c1-200
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $D/pytest_w2.log | head -20 | cut -c1-300; exit $rc; }
for w2 in 0 1; do
  MANDO_POA_W2=$w2 timeout -k 10 400 python3 bench.py --no-cpu-baseline --workload config5 --steps 2 --warmup 1 > $D/bench_c5_w$w2.json 2> $D/bench_c5_w$w2.err || { echo "c5 w2=$w2 failed"; tail -5 $D/bench_c5_w$w2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_c5_w$w2.json')); c=d['config']; print('c5 w2=$w2', round(d['ms_per_step'], 1), c['steps_poa_kernel_ms'], c.get('full_output_equals_oracle'))"
done
