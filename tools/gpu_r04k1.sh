# GPU box: K1 line scan / tab scan change -- GPU tests (all with FULL=1), smoke, config-2 phases,
# config 2 / 3 / 4 benches (full-output hashes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04k1}
mkdir -p $D
T=tests/test_cluster_gpu.py; [ -n "$FULL" ] && T=tests
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread $T > $D/pytest.log 2>&1 || { tail -20 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
if [ -n "$FULL" ]; then timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }; tail -1 $D/smoke.log; fi
MANDO_LIB=variants/clph/libmando.so MANDO_CL_TIME=1 timeout -k 10 300 python3 bench.py --workload config2 --steps 1 --warmup 0 --no-cpu-baseline > $D/c2ph.out 2> $D/c2ph.err || { tail -20 $D/c2ph.err; exit 1; }
grep -h "cluster\]\|K1 phases" $D/c2ph.err $D/c2ph.out
for w in config2 config3 ${C4:-}; do
  st=5; [ $w = config4 ] && st=3
  MANDO_CL_TIME=1 timeout -k 10 600 python3 bench.py --workload $w --steps $st --warmup 1 --no-cpu-baseline > $D/$w.json 2> $D/$w.err || { tail -20 $D/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$w.json')); c=d['config']; print('$w', round(d['ms_per_step'],1), round(d['value']), c['full_output_equals_oracle'], c['steps_s'], c['phases_rank0_s']['t_cluster'])"
done
