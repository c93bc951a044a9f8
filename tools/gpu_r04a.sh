# GPU box, round 4 first call: the new driver tests (explicit POA budget, metrics line), the cross-wave
# exchange micro-benchmark, and config 4 at HEAD with the HBM-plan calibration log (MANDO_WS_LOG).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r04a
mkdir -p $D
timeout -k 10 60 ./tools/ubench_xwave > $D/ubench_xwave.txt 2>&1 && cat $D/ubench_xwave.txt || exit 1
timeout -k 10 600 python -u -m pytest tests/test_define_gpu.py tests/test_mando_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; grep -E "passed|failed" $D/pytest.log | tail -2 | cut -c1-200
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $D/pytest.log | head -20 | cut -c1-300; exit $rc; }
MANDO_WS_LOG=1 timeout -k 10 900 python3 bench.py --no-cpu-baseline --workload config4 --steps 1 --warmup 0 > $D/bench_config4.json 2> $D/bench_config4.err || { echo "config4 failed"; tail -5 $D/bench_config4.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_config4.json')); print('config4', d['value'], round(d['ms_per_step'], 1), d['config']['phases_rank0_s'])"
grep -c "mando ws" $D/bench_config4.err
