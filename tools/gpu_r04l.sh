# GPU box: config 3 with the clustering phase breakdown (MANDO_CL_TIME) and the timeline; config 4 N=1 and
# the 2/4/8-rank rehearsals at HEAD (two-wave wide groups on, workspace headroom).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04l}
mkdir -p $D
MANDO_CL_TIME=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $D/bench_config3.json 2> $D/bench_config3.err || { tail -5 $D/bench_config3.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_config3.json')); c=d['config']; print('config3', round(d['value']), round(d['ms_per_step'], 1), c['steps_s'], c['phases_rank0_s'], c.get('full_output_equals_oracle'))"
grep "\[cluster\]" $D/bench_config3.err | tail -4
timeout -k 10 300 python3 tools/e2e_timeline.py 20000 > $D/timeline.txt 2>&1 && tail -9 $D/timeline.txt || exit 1
timeout -k 10 900 python3 bench.py --no-cpu-baseline --workload config4 --steps 2 --warmup 1 > $D/bench_config4.json 2> $D/bench_config4.err || { tail -5 $D/bench_config4.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_config4.json')); c=d['config']; print('config4', round(d['value']), round(d['ms_per_step'], 1), c['steps_s'], c['phases_rank0_s'])"
for n in 2 4 8; do
  timeout -k 10 600 python3 tools/rank_rehearsal.py /tmp/mando_bench_config4_200000 $n 16 > $D/rehearsal_config4_$n.json 2> $D/rehearsal_config4_$n.err || { echo "rehearsal $n failed"; tail -5 $D/rehearsal_config4_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/rehearsal_config4_$n.json')); print('rehearsal config4', $n, d['rank_s'], d['rank0_phases_s'], 'pred', d['predicted_step_s'], 'eq', d['reassembled_equals_one_rank'])"
done
