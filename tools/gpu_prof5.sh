# GPU box: per-phase POA cycle counters (MANDO_PROF=1) on the config-5 (-S) and config-2 workloads.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-p5}
mkdir -p $D
export TMPDIR=/tmp
for w in ${WLS:-config5 config2}; do
  MANDO_PROF=1 timeout -k 10 300 python bench.py --workload $w --steps 1 --warmup 0 --no-cpu-baseline > $D/$w.json 2> $D/$w.err || { echo "$w failed"; tail -20 $D/$w.err; exit 1; }
  grep "mando prof" $D/$w.err | cut -c1-250; python3 -c "import json,sys; d=json.load(open('$D/$w.json')); print('$w', d['ms_per_step'], d['config']['phases_rank0_s'], d['config']['poa_kernel'])"
done
