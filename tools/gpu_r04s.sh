# GPU box: where the clustering phase goes (MANDO_CL_TIME=1: file sizes, reads + copy, K1, K2, flatten) on
# config 3 and on an 8-rank config-4 share; and config 4 on one GPU with the POA grids capped below 16
# waves per CU (wave slots left to the next chunk's clustering / orientation kernels).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04s}
mkdir -p $D
MANDO_CL_TIME=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload config3 --steps 3 --warmup 1 > $D/c3_cltime.json 2> $D/c3_cltime.err || { echo c3 failed; tail -5 $D/c3_cltime.err; exit 1; }
grep -i "cluster\|K1\|K2" $D/c3_cltime.err | tail -12
MANDO_CL_TIME=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload config4 --share 8 --steps 3 --warmup 1 > $D/c4s8_cltime.json 2> $D/c4s8_cltime.err || { echo c4s8 failed; tail -5 $D/c4s8_cltime.err; exit 1; }
grep -i "cluster\|K1\|K2" $D/c4s8_cltime.err | tail -8
run() {  # name, env assignments...
  local name=$1; shift
  env "$@" timeout -k 10 600 python3 bench.py --no-cpu-baseline --workload config4 --steps 3 --warmup 1 > $D/$name.json 2> $D/$name.err || { echo "$name failed"; tail -5 $D/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$name.json')); c=d['config']; print('$name', round(d['ms_per_step'], 1), c['steps_s'], c['steps_poa_kernel_ms'], c['phases_rank0_s'])"
}
run c4_w16 MANDO_X=0 || exit 1
run c4_w15 MANDO_POA_OCC=15 || exit 1
run c4_w14 MANDO_POA_OCC=14 || exit 1
