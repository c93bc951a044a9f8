# GPU box: default bench line (config 3) plus config 5 / config 2 steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-b3}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --no-cpu-baseline ${BARGS:-} > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$D/bench.json')); print('config3', d['ms_per_step'], d['config']['phases_rank0_s'], d['config']['poa_kernel'])"
for w in ${WLS:-config5 config2}; do
  timeout -k 10 400 python bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline > $D/$w.json 2> $D/$w.err || { echo "$w failed"; tail -20 $D/$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$D/$w.json')); print('$w', d['ms_per_step'], d['config']['phases_rank0_s'], d['config']['poa_kernel'])"
done
