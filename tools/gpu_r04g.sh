# GPU box: comm + driver GPU tests; config 3 and config 4 at N=1 (phase times incl. the output writes);
# the per-rank loads of 2/4/8-rank LPT plans (bench.py --share), each alone on this GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04g}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_comm.py tests/test_define_ref.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; grep -E "passed|failed" $D/pytest.log | tail -2 | cut -c1-200
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $D/pytest.log | head -20 | cut -c1-300; exit $rc; }
for w in config3 config4; do
  st=3; [ $w = config4 ] && st=1
  timeout -k 10 900 python3 bench.py --no-cpu-baseline --workload $w --steps $st --warmup 1 > $D/bench_$w.json 2> $D/bench_$w.err || { echo "$w failed"; tail -5 $D/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$w.json')); c=d['config']; print('$w N=1', round(d['value']), round(d['ms_per_step'], 1), c['chunks'], c['phases_rank0_s'], c.get('full_output_equals_oracle'))"
  for n in 2 4 8; do
    st=2; [ $w = config3 ] && st=4
    timeout -k 10 600 python3 bench.py --workload $w --share $n --steps $st --warmup 1 > $D/share_${w}_$n.json 2> $D/share_${w}_$n.err || { echo "share $w $n failed"; tail -5 $D/share_${w}_$n.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/share_${w}_$n.json')); c=d['config']; print('share $w 1/$n', c['records'], round(d['ms_per_step'], 1), c['steps_s'], c['phases_rank0_s'])"
  done
done
