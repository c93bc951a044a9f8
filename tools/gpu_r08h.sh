# A/B of one hardware queue per library stream (default) against HIP's shared queues
# (MANDO_SHARED_QUEUES=1), config 4 on one GPU, interleaved, 3 steps + 1 warmup; then a kernel trace of
# one step with the default.  (r08i / r08j ran the same script with a stream-priority knob in place of
# MANDO_SHARED_QUEUES, since removed: profiles/r08h_ab_queues.txt.)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08h}
mkdir -p $D
run() {
  env MANDO_SHARED_QUEUES=$2 timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $D/$1.json 2> $D/$1.err || { echo "$1 failed"; tail -5 $D/$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$1.json')); c=d['config']; print('$1', round(d['ms_per_step']), c['steps_s'], c['steps_poa_kernel_ms'], c['full_output_equals_oracle'])" | tee -a $D/summary.txt
}
for i in 1 2; do
  run own.$i 0 && run shared.$i 1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o trace -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > $D/trace_bench.json 2> $D/trace_bench.err || { echo "trace failed"; tail -5 $D/trace_bench.err; exit 1; }
echo done
