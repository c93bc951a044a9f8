# GPU box: config 4 and config 3 at N=1 (one vs two waves per wide group), then the N-rank rehearsal on
# one GPU (tools/rank_rehearsal.py): every rank's share in turn, rank 0's merge + write of the whole
# output, and the reassembled files against the one-rank run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04h}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_define_ref.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -1 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in config4 config3; do
  for w2 in 1; do
    st=2; [ $w = config3 ] && st=4
    MANDO_POA_W2=$w2 timeout -k 10 900 python3 bench.py --no-cpu-baseline --workload $w --steps $st --warmup 1 > $D/bench_${w}_w$w2.json 2> $D/bench_${w}_w$w2.err || { echo "$w failed"; tail -5 $D/bench_${w}_w$w2.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/bench_${w}_w$w2.json')); c=d['config']; print('$w N=1 w2=$w2', round(d['value']), round(d['ms_per_step'], 1), c['steps_s'], c['phases_rank0_s'], c.get('full_output_equals_oracle'))"
  done
  for n in 2 4 8; do
    timeout -k 10 600 python3 tools/rank_rehearsal.py /tmp/mando_bench_${w}_$([ $w = config4 ] && echo 200000 || echo 20000) $n 16 > $D/rehearsal_${w}_$n.json 2> $D/rehearsal_${w}_$n.err || { echo "rehearsal $w $n failed"; tail -5 $D/rehearsal_${w}_$n.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/rehearsal_${w}_$n.json')); print('rehearsal $w', $n, d['rank_s'], d['rank0_phases_s'], 'pred', d['predicted_step_s'], 'eq', d['reassembled_equals_one_rank'])"
  done
done
