# GPU box: one GPU running the per-rank share of a strong-scaling config-3 run (20,000 / N loci for
# N = 2, 4, 8): the step time each rank would need before the all-gather, i.e. an upper bound on the
# driver's 1 -> N scaling; the N = 8 share also with one chunk (MANDO_CHUNKS=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-share}
mkdir -p $D
run() {
  env $3 timeout -k 10 300 python3 bench.py --loci $2 --steps 5 --warmup 1 --no-cpu-baseline > $D/$1.json 2> $D/$1.err || { echo "$1 failed"; tail -5 $D/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$D/$1.json')); c=d['config']; print('$1', round(d['ms_per_step'], 1), c['steps_s'], c['phases_rank0_s'])"
}
run loci10000 10000 "" && run loci5000 5000 "" && run loci2500 2500 "" && run loci2500_1chunk 2500 "MANDO_CHUNKS=1" && run loci2500_3chunks 2500 "MANDO_CHUNKS=3"
