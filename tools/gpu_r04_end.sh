# GPU box, round 4 end: the rocprofv3 PMC (FETCH_SIZE, WRITE_SIZE), kernel-trace and SQ passes of the default
# bench (config 4; tools/profile_round.sh) and bench lines for configs 2, 3 and 5.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r04y}
MANDO_COMMIT=${MANDO_COMMIT:-unknown} WL=config4 TAG=${T}_prof bash tools/profile_round.sh || exit 1
D=gpurun_out/${T}
mkdir -p $D
for w in config2 config3 config5; do
  timeout -k 10 500 python3 bench.py --workload $w --no-cpu-baseline > $D/bench_$w.json 2> $D/bench_$w.err || { echo "$w failed"; tail -20 $D/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$w.json')); c=d['config']; print('$w', round(d['ms_per_step'], 1), c['steps_s'], c['phases_rank0_s'], c.get('full_output_equals_oracle'))"
done
