# GPU box: config-3 bench lines for several (source tree, environment) variants -- trees are this one (.)
# or git worktrees of older commits under _wt/, each built in the container -- interleaved twice.
# usage: bash tools/gpu_ab_trees.sh TAG "name|dir|ENV=1 ENV2=x" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$PWD
D=$R/gpurun_out/${1:-abt}
shift
mkdir -p $D
export TMPDIR=/tmp
for pass in 1 2; do
  for v in "$@"; do
    n=${v%%|*}; rest=${v#*|}; t=${rest%%|*}; envs=${rest#*|}; [ "$envs" = "$rest" ] && envs=""
    (cd $t && env $envs timeout -k 10 400 python3 bench.py --steps ${STEPS:-6} --warmup 1 --no-cpu-baseline --data-dir /tmp/abt_data ${BARGS:-} > $D/$n.$pass.json 2> $D/$n.$pass.err) || { echo "$n failed"; tail -5 $D/$n.$pass.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/$n.$pass.json')); c=d['config']; print('$n.$pass', round(d['ms_per_step'],1), c['steps_s'], c.get('steps_poa_kernel_ms'), c['phases_rank0_s']['t_cluster'], c.get('full_output_equals_oracle'))"
  done
done
