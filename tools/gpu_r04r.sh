# GPU box: config 4 on one GPU (16 chunks of 4 GiB): one POA stream (default) against two (chunk k+1's
# launches beside chunk k's tail), and 8 GiB chunks with two streams; interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04r}
mkdir -p $D
run() {  # name, env assignments...
  local name=$1; shift
  env "$@" timeout -k 10 600 python3 bench.py --no-cpu-baseline --workload config4 --steps 3 --warmup 1 > $D/$name.json 2> $D/$name.err || { echo "$name failed"; tail -5 $D/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$name.json')); c=d['config']; print('$name', round(d['ms_per_step'], 1), c['steps_s'], c['steps_poa_kernel_ms'], c['phases_rank0_s'], c.get('chunks'), c.get('full_output_equals_oracle'))"
}
for rep in 1 2; do
  run c4n1_s1_$rep MANDO_X=0 || exit 1
  run c4n1_s2_$rep MANDO_POA_STREAMS=2 || exit 1
  run c4n1_8g_s2_$rep MANDO_POA_STREAMS=2 MANDO_CHUNK_BYTES=8589934592 || exit 1
done
