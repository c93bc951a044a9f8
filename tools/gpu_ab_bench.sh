# GPU box: bench.py lines (config 3, STEPS steps) for several libmando builds, interleaved twice.
# usage: bash tools/gpu_ab_bench.sh TAG name=path/to/libmando.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-abb}
shift
mkdir -p $D
export TMPDIR=/tmp
for pass in 1 2; do
  for kv in "$@"; do
    n=${kv%%=*}; lib=${kv#*=}
    MANDO_LIB=$lib timeout -k 10 400 python3 bench.py --steps ${STEPS:-8} --warmup 1 --no-cpu-baseline ${BARGS:-} > $D/$n.$pass.json 2> $D/$n.$pass.err || { echo "$n failed"; tail -5 $D/$n.$pass.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/$n.$pass.json')); c=d['config']; print('$n.$pass', round(d['ms_per_step'],1), c['steps_s'], c['steps_poa_kernel_ms'], c['full_output_equals_oracle'])"
  done
done
