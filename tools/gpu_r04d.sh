# GPU box: config-3 stage timelines -- one chunk, heaviest-first, heaviest-first with 8 hardware queues --
# then config 4 at HEAD (HBM plan with the calibrated reserve).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04d}
mkdir -p $D
MANDO_HEAVY_FRAC=0 timeout -k 10 300 python3 tools/e2e_timeline.py 20000 > $D/tl_one.txt 2>&1 && tail -9 $D/tl_one.txt || exit 1
timeout -k 10 300 python3 tools/e2e_timeline.py 20000 > $D/tl_heavy.txt 2>&1 && tail -14 $D/tl_heavy.txt || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 tools/e2e_timeline.py 20000 > $D/tl_heavy_q8.txt 2>&1 && tail -14 $D/tl_heavy_q8.txt || exit 1
MANDO_WS_LOG=1 timeout -k 10 900 python3 bench.py --no-cpu-baseline --workload config4 --steps 1 --warmup 0 > $D/bench_config4.json 2> $D/bench_config4.err || { echo "config4 failed"; tail -5 $D/bench_config4.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_config4.json')); print('config4', d['value'], round(d['ms_per_step'], 1), d['config']['phases_rank0_s'])"
