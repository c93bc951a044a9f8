# GPU box: config-3 bench (12 steps) with the per-workgroup placement / timing trace of every one-group POA
# launch (MANDO_WG_TRACE), summarised per launch (tools/wg_trace.py).  The probe is not in the product
# sources: apply tools/wg_trace_probe.patch (git apply) and rebuild first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-wgt}
mkdir -p $D
rm -f $D/trace.txt
MANDO_WG_TRACE=$D/trace.txt timeout -k 10 400 python3 bench.py --steps 12 --warmup 1 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -5 $D/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench.json')); c=d['config']; print(c['steps_s']); print(c['steps_poa_kernel_ms'])"
python3 tools/wg_trace.py $D/trace.txt > $D/summary.txt && cat $D/summary.txt
