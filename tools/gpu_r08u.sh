# Wide groups as their own batch with four chunks in flight (define.py defaults) against one batch per
# chunk with three in flight (MANDO_SPLIT_WIDE=0 MANDO_INFLIGHT=3): config 4, 20 steps + 3 warmup each.
# ORDER="new base" or "base new"; TESTS=1 runs the GPU tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08u}
mkdir -p $D
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_split_wide.py tests/test_define_gpu.py tests/test_poa_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest.log | cut -c1-300
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $D/pytest.log | head -30 | cut -c1-300; exit $rc; }
fi
for v in ${ORDER:-new base}; do
  if [ $v = new ]; then E="MANDO_SPLIT_WIDE=1 MANDO_INFLIGHT=4"; else E="MANDO_SPLIT_WIDE=0 MANDO_INFLIGHT=3"; fi
  N=$v.$(date +%s)
  env $E timeout -k 10 560 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $D/$N.json 2> $D/$N.err || { echo "$N failed"; tail -5 $D/$N.err; exit 1; }
  python3 -c "import json,statistics as s; d=json.load(open('$D/$N.json')); c=d['config']; x=c['steps_s']; print('$v', round(d['ms_per_step']), 'median', round(s.median(x),3), 'max', max(x), c['full_output_equals_oracle'])" | tee -a $D/summary.txt
done
