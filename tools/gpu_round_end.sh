# GPU box, end of a round: every GPU test, smoke, the default bench line and timeline (gpu_full.sh), the
# rocprofv3 PMC / kernel-trace / SQ passes of the default bench (profile_round.sh), and bench lines for
# configs 2 and 5.  usage: TAG=r02j bash tools/gpu_round_end.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-re}
RUN=${T} bash tools/gpu_full.sh || exit 1
TAG=${T}_prof bash tools/profile_round.sh || exit 1
D=gpurun_out/${T}
for w in config2 config5; do
  timeout -k 10 500 python bench.py --workload $w --no-cpu-baseline > $D/bench_$w.json 2> $D/bench_$w.err || { echo "$w failed"; tail -20 $D/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$w.json')); print('$w', round(d['ms_per_step'], 1), d['config']['phases_rank0_s'])"
done
