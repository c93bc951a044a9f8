# GPU box: a 12-step config-3 bench under rocprofv3 --kernel-trace (slow-step forensics: which POA launch
# stretches and what runs beside it).  usage: RUN=r03o bash tools/gpu_slowsteps.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-slow}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $D/kt -o kt --output-format csv -- python3 bench.py --steps ${STEPS:-12} --warmup 1 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench.json')); print(d['ms_per_step'], d['config']['steps_s'], d['config']['steps_poa_kernel_ms'])"
F=$(find $D/kt -name "*kernel_trace.csv" | head -1)
python3 tools/slow_steps.py $F > $D/slow_steps.txt 2>&1; tail -40 $D/slow_steps.txt
