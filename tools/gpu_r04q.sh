# GPU box: an 8-rank share (rank 0's loci of the LPT plan, alone on one GPU) of config 4 and of config 3,
# one chunk (the default below 8 GB) against pipelined chunks (clustering and orientation of chunk k+1
# beside the POA of chunk k), with one and two POA streams; and the heavy-group wave priority.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04q}
mkdir -p $D
run() {  # name, workload, env assignments...
  local name=$1 w=$2; shift 2
  env "$@" timeout -k 10 600 python3 bench.py --no-cpu-baseline --workload $w --share 8 --steps 5 --warmup 2 > $D/$name.json 2> $D/$name.err || { echo "$name failed"; tail -5 $D/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$name.json')); c=d['config']; print('$name', round(d['ms_per_step'], 1), c['steps_s'], c['steps_poa_kernel_ms'], c['phases_rank0_s'], c.get('chunks'))"
}
for rep in 1 2; do
  run c4_one_$rep config4 MANDO_X=0 || exit 1
  run c4_ch4_$rep config4 MANDO_TWO_CHUNK_BYTES=536870912 MANDO_CHUNK_BYTES=268435456 || exit 1
  run c4_ch4s2_$rep config4 MANDO_TWO_CHUNK_BYTES=536870912 MANDO_CHUNK_BYTES=268435456 MANDO_POA_STREAMS=2 || exit 1
  run c4_ch2s2_$rep config4 MANDO_CHUNKS=2 MANDO_FIRST_CHUNK=0.3 MANDO_POA_STREAMS=2 || exit 1
  run c4_hp_$rep config4 MANDO_POA_HEAVY_PRIO=0.5 || exit 1
done
for rep in 1 2; do
  run c3_one_$rep config3 MANDO_X=0 || exit 1
  run c3_ch2s2_$rep config3 MANDO_CHUNKS=2 MANDO_FIRST_CHUNK=0.3 MANDO_POA_STREAMS=2 || exit 1
  run c3_hp5_$rep config3 MANDO_POA_HEAVY_PRIO=0.5 || exit 1
  run c3_hp2_$rep config3 MANDO_POA_HEAVY_PRIO=0.2 || exit 1
done
