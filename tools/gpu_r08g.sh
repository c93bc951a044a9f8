# 2/4/8-rank rehearsals of config 4 at HEAD (reader cap in force), after one one-rank step that leaves
# the reference files the rehearsals hash against.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08g}
mkdir -p $D
DATA=/tmp/mando_bench_config4_200000
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -5 $D/bench.err; exit 1; }
for spec in "2 8" "4 4" "8 2" "8 16"; do
  set -- $spec
  timeout -k 10 400 python3 tools/rank_rehearsal.py $DATA $1 $2 > $D/rehearsal_config4_$1_t$2.json 2> $D/rehearsal_$1_$2.err || { echo "rehearsal $1 $2 failed"; tail -5 $D/rehearsal_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/rehearsal_config4_$1_t$2.json')); print('$1 ranks, $2 threads:', d['rank_s'], d['predicted_step_s'], d['reassembled_equals_one_rank'])"
done
