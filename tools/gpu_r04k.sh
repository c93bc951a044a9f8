# GPU box: smaller first-attempt kp/spill capacities -- POA parity tests, config 3/5/4 with the workspace
# log (slot sizes, capacity re-runs), then the config-4 8-rank rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04k}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_poa_gpu.py tests/test_define_gpu.py tests/test_abpoa_cli.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -1 $D/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $D/pytest.log | head; exit $rc; }
for w in config3 config5 config4; do
  st=3; [ $w = config4 ] && st=2
  MANDO_WS_LOG=1 timeout -k 10 900 python3 bench.py --no-cpu-baseline --workload $w --steps $st --warmup 1 > $D/bench_$w.json 2> $D/bench_$w.err || { echo "$w failed"; tail -5 $D/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$w.json')); c=d['config']; print('$w N=1', round(d['value']), round(d['ms_per_step'], 1), c['steps_s'], c['steps_poa_kernel_ms'], c.get('full_output_equals_oracle'))"
  grep -E "re-run|slot workspace" $D/bench_$w.err | sort | uniq -c | sort -rn | head -4 | cut -c1-180
done
timeout -k 10 600 python3 tools/rank_rehearsal.py /tmp/mando_bench_config4_200000 8 16 > $D/rehearsal_config4_8.json 2> $D/rehearsal_config4_8.err || { echo "rehearsal failed"; tail -5 $D/rehearsal_config4_8.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/rehearsal_config4_8.json')); print('rehearsal config4 8', d['rank_s'], d['rank0_phases_s'], 'pred', d['predicted_step_s'], 'eq', d['reassembled_equals_one_rank'])"
