# GPU box, round 4: heaviest-first pipeline + two-wave wide groups.  Parity tests first (bounded), then a
# config-3 A/B (one chunk vs heaviest-first, one vs two waves per wide group), then config 4 at HEAD with
# the HBM-plan calibration log (MANDO_WS_LOG).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04c}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_define_ref.py tests/test_define_gpu.py tests/test_mando_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; grep -E "passed|failed" $D/pytest.log | tail -2 | cut -c1-200
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $D/pytest.log | head -20 | cut -c1-300; exit $rc; }
B="python3 bench.py --no-cpu-baseline --steps 4 --warmup 1"
for pass in 1 2; do
  for v in "0 0" "0.3 0" "0.3 1"; do
    set -- $v
    MANDO_HEAVY_FRAC=$1 MANDO_POA_W2=$2 timeout -k 10 300 $B > $D/c3_h$1_w$2_$pass.json 2> $D/c3_h$1_w$2_$pass.err || { echo "c3 $v failed"; tail -5 $D/c3_h$1_w$2_$pass.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/c3_h$1_w$2_$pass.json')); c=d['config']; print('c3 heavy=$1 w2=$2', round(d['ms_per_step'], 1), c['steps_s'], c['steps_poa_kernel_ms'], c['phases_rank0_s'], c.get('full_output_equals_oracle'))"
  done
done
MANDO_WS_LOG=1 timeout -k 10 900 python3 bench.py --no-cpu-baseline --workload config4 --steps 1 --warmup 0 > $D/bench_config4.json 2> $D/bench_config4.err || { echo "config4 failed"; tail -5 $D/bench_config4.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_config4.json')); print('config4', d['value'], round(d['ms_per_step'], 1), d['config']['phases_rank0_s'])"
grep "mando ws" $D/bench_config4.err | sort | uniq -c | sort -rn | head -5 | cut -c1-200
