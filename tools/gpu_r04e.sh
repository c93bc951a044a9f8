# GPU box: POA + driver parity tests, config-3 one-chunk A/B (one vs two waves per wide group, interleaved),
# config 4 at HEAD (per-kind workspace grants, backpressure).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04e}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_poa_gpu.py tests/test_define_ref.py tests/test_define_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; grep -E "passed|failed" $D/pytest.log | tail -2 | cut -c1-200
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $D/pytest.log | head -20 | cut -c1-300; exit $rc; }
B="python3 bench.py --no-cpu-baseline --steps 5 --warmup 1"
for pass in 1 2; do
  for w2 in 0 1; do
    MANDO_POA_W2=$w2 timeout -k 10 300 $B > $D/c3_w${w2}_$pass.json 2> $D/c3_w${w2}_$pass.err || { echo "c3 w2=$w2 failed"; tail -5 $D/c3_w${w2}_$pass.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/c3_w${w2}_$pass.json')); c=d['config']; print('c3 w2=$w2', round(d['ms_per_step'], 1), c['steps_s'], c['steps_poa_kernel_ms'], c.get('full_output_equals_oracle'))"
  done
done
MANDO_WS_LOG=1 timeout -k 10 900 python3 bench.py --no-cpu-baseline --workload config4 --steps 1 --warmup 0 > $D/bench_config4.json 2> $D/bench_config4.err || { echo "config4 failed"; tail -5 $D/bench_config4.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_config4.json')); print('config4', d['value'], round(d['ms_per_step'], 1), d['config']['phases_rank0_s'])"
