# GPU box: warm config-5 / config-2 bench steps with the stage split (MANDO_PROF=1 optional).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-c5}
mkdir -p $D
export TMPDIR=/tmp
for w in ${WLS:-config5}; do
  timeout -k 10 400 python bench.py --workload $w --steps ${STEPS:-1} --warmup 1 --no-cpu-baseline > $D/$w.json 2> $D/$w.err || { echo "$w failed"; tail -20 $D/$w.err; exit 1; }
  grep "mando" $D/$w.err | cut -c1-250 | tail -30; python3 -c "import json,sys; d=json.load(open('$D/$w.json')); print('$w', d['ms_per_step'], d['config']['phases_rank0_s'], d['config']['poa_kernel'])"
done
