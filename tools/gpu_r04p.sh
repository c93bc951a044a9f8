# GPU box: A/B of the heavy-group wave priority (MANDO_POA_HEAVY_PRIO: groups within that fraction of the
# launch's largest DP-cost estimate run two priority levels higher) on an 8-rank config-3 share (the POA
# floor of a multi-GPU step: its longest group) and on the whole config 3; interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04p}
mkdir -p $D
run() {  # name, env value, extra args
  MANDO_POA_HEAVY_PRIO=$2 timeout -k 10 600 python3 bench.py --no-cpu-baseline --workload config3 $3 > $D/$1.json 2> $D/$1.err || { echo "$1 failed"; tail -5 $D/$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$1.json')); c=d['config']; print('$1', round(d['ms_per_step'], 1), c['steps_poa_kernel_ms'], c['phases_rank0_s']['t_poa'])"
}
for rep in 1 2; do
  for h in 0 0.5 0.2; do
    run share8_h${h}_$rep $h "--share 8 --steps 6 --warmup 2" || exit 1
  done
done
for rep in 1 2; do
  for h in 0 0.5; do
    run full_h${h}_$rep $h "--steps 4 --warmup 1" || exit 1
  done
done
