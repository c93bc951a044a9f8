# GPU box: the multi-GPU prediction at HEAD -- config 3 and config 4 at N=1 and the 2/4/8-rank rehearsals
# (each rank's share warmed, then timed; rank 0 merges and writes the whole output).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04n}
mkdir -p $D
for w in ${WS:-config3 config4}; do
  st=3; [ $w = config4 ] && st=2
  timeout -k 10 900 python3 bench.py --no-cpu-baseline --workload $w --steps $st --warmup 1 > $D/bench_$w.json 2> $D/bench_$w.err || { echo "$w failed"; tail -5 $D/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$w.json')); c=d['config']; print('$w N=1', round(d['value']), round(d['ms_per_step'], 1), c['steps_s'], c['phases_rank0_s'], c.get('full_output_equals_oracle'))"
  for n in 2 4 8; do
    timeout -k 10 900 python3 tools/rank_rehearsal.py /tmp/mando_bench_${w}_$([ $w = config4 ] && echo 200000 || echo 20000) $n 16 > $D/rehearsal_${w}_$n.json 2> $D/rehearsal_${w}_$n.err || { echo "rehearsal $w $n failed"; tail -5 $D/rehearsal_${w}_$n.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/rehearsal_${w}_$n.json')); print('rehearsal $w', $n, d['rank_s'], d.get('rank_phases_s', {}).get('0', d.get('rank0_phases_s')), 'pred', d['predicted_step_s'], d.get('predicted_step_serial_fasta_s'), 'eq', d['reassembled_equals_one_rank'])"
  done
done
