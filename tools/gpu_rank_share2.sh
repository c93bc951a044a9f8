# GPU box: per-rank shares of the config-3 strong-scaling run with one chunk against two (see
# tools/gpu_rank_share.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-share2}
mkdir -p $D
run() {
  env $3 timeout -k 10 300 python3 bench.py --loci $2 --steps 4 --warmup 1 --no-cpu-baseline > $D/$1.json 2> $D/$1.err || { echo "$1 failed"; tail -5 $D/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$D/$1.json')); c=d['config']; print('$1', round(d['ms_per_step'], 1), c['steps_s'], c['phases_rank0_s'])"
}
run l5000_1c 5000 "MANDO_CHUNKS=1" && run l10000_1c 10000 "MANDO_CHUNKS=1" && run l10000_f02 10000 "MANDO_FIRST_CHUNK=0.2" && run l20000_1c 20000 "MANDO_CHUNKS=1" && run l20000_f02 20000 "MANDO_FIRST_CHUNK=0.2" && run l20000 20000 ""
