# GPU box: config-3 bench lines for several chunk splits (MANDO_CHUNK_FRACS, cumulative byte fractions).
# usage: bash tools/gpu_chunks_ab.sh TAG "0.3" "0.25,0.6" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-chunks}
shift
mkdir -p $D
export TMPDIR=/tmp
for pass in 1 2; do
  for fr in "$@"; do
    n=$(echo $fr | tr ',' '_')
    MANDO_CHUNK_FRACS=$fr timeout -k 10 400 python3 bench.py --steps ${STEPS:-6} --warmup 1 --no-cpu-baseline > $D/$n.$pass.json 2> $D/$n.$pass.err || { echo "$fr failed"; tail -5 $D/$n.$pass.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/$n.$pass.json')); c=d['config']; print('$fr.$pass', round(d['ms_per_step'],1), c['steps_s'], c['steps_poa_kernel_ms'], c['full_output_equals_oracle'])"
  done
done
