# GPU box: bench lines of the other workloads (config 2 SIRV-like, config 5 long / -S), default pipeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-c25}; mkdir -p $D
export TMPDIR=/tmp
for w in config2 config5; do
  timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $D/$w.json 2> $D/$w.err || { tail -5 $D/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$w.json')); print('$w', round(d['ms_per_step']), d['config']['phases_rank0_s'])"
done
