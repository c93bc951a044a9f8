# GPU box: full validation (tests, smoke, default bench, timeline) + config-5 POA profile lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_full.sh || exit 1
D=gpurun_out/${RUN:-full}
MANDO_PROF=1 timeout -k 10 400 python bench.py --workload config5 --steps 1 --warmup 0 --no-cpu-baseline > $D/c5.json 2> $D/c5.err || { echo "c5 failed"; tail -20 $D/c5.err; exit 1; }
grep "mando prof" $D/c5.err | grep -E "fast rows|slots=|team" | cut -c1-160
