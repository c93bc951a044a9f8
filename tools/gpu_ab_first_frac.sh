# A/B of the first chunk's share of a config-4 chunk (MANDO_FIRST_FRAC), interleaved, 3 steps + 1 warmup.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-abff}
mkdir -p $D
run() {
  env MANDO_FIRST_FRAC=$2 timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $D/$1.json 2> $D/$1.err || { echo "$1 failed"; tail -5 $D/$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$1.json')); c=d['config']; print('$1', round(d['ms_per_step']), c['steps_s'], c['steps_poa_kernel_ms'], c['full_output_equals_oracle'])" | tee -a $D/summary.txt
}
for i in 1 2; do
  run f40.$i 0.4 && run f20.$i 0.2 && run f28.$i 0.28 || exit 1
done
