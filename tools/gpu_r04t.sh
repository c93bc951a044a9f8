# GPU box: config 4 on one GPU (16 chunks) with the POA streams leaving the first k CUs to the next
# chunk's clustering / orientation kernels (MANDO_POA_FREE_CUS, hipExtStreamCreateWithCUMask), k = 0 / 16 /
# 32 / 48, interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04t}
mkdir -p $D
run() {  # name, env assignments...
  local name=$1; shift
  env "$@" timeout -k 10 600 python3 bench.py --no-cpu-baseline --workload config4 --steps 3 --warmup 1 > $D/$name.json 2> $D/$name.err || { echo "$name failed"; tail -5 $D/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$name.json')); c=d['config']; print('$name', round(d['ms_per_step'], 1), c['steps_s'], c['steps_poa_kernel_ms'], c['phases_rank0_s'], c.get('full_output_equals_oracle'))"
}
for rep in 1 2; do
  for k in 0 32 16 48; do
    run c4_free${k}_$rep MANDO_POA_FREE_CUS=$k || exit 1
  done
done
