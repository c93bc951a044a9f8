# GPU box: 16-row descriptor batches + the -S leader state in dynamic LDS (narrow launches at 16 waves per
# CU): POA parity tests, then an interleaved A/B against 32-row batches (POA per-row cycles on 20,000
# config-3 groups, and the config-3 bench).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04m}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_poa_gpu.py tests/test_abpoa_cli.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -1 $D/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $D/pytest.log | head; exit $rc; }
bash tools/ab_prof.sh r04m_ab d16=variants/desc16/libmando.so d32=variants/desc32/libmando.so || exit 1
for pass in 1 2; do
  for v in desc16 desc32; do
    MANDO_WS_LOG=1 MANDO_LIB=variants/$v/libmando.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 4 --warmup 1 > $D/c3_${v}_$pass.json 2> $D/c3_${v}_$pass.err || { tail -3 $D/c3_${v}_$pass.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/c3_${v}_$pass.json')); c=d['config']; print('c3 $v', round(d['ms_per_step'], 1), c['steps_s'], c['steps_poa_kernel_ms'], c.get('full_output_equals_oracle'))"
    grep -m2 "waves per CU" $D/c3_${v}_$pass.err | tail -1 | cut -c1-120
  done
done
