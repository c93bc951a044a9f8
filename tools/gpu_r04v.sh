# GPU box: orientation inside the clustering call (each sub-batch oriented beside the next one's
# clustering; default) against the separate orientation call after it (MANDO_ORIENT_IN_CLUSTER=0): the
# clustering / define GPU tests, then config 3 and an 8-rank config-4 share, interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04v}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_cluster_gpu.py tests/test_define_ref.py tests/test_orient.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
run() {  # name, workload args, env assignments...
  local name=$1 wl=$2; shift 2
  env "$@" timeout -k 10 600 python3 bench.py --no-cpu-baseline $wl > $D/$name.json 2> $D/$name.err || { echo "$name failed"; tail -5 $D/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$name.json')); c=d['config']; print('$name', round(d['ms_per_step'], 1), c['steps_s'], c['phases_rank0_s'], c.get('full_output_equals_oracle'))"
}
for rep in 1 2; do
  run c3_in_$rep "--workload config3 --steps 5 --warmup 1" MANDO_X=0 || exit 1
  run c3_sep_$rep "--workload config3 --steps 5 --warmup 1" MANDO_ORIENT_IN_CLUSTER=0 || exit 1
  run c4s8_in_$rep "--workload config4 --share 8 --steps 4 --warmup 1" MANDO_X=0 || exit 1
  run c4s8_sep_$rep "--workload config4 --share 8 --steps 4 --warmup 1" MANDO_ORIENT_IN_CLUSTER=0 || exit 1
done
run c4_in "--workload config4 --steps 3 --warmup 1" MANDO_X=0 || exit 1
