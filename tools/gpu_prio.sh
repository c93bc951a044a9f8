# GPU box: POA parity, then config-3 bench lines with and without the wide launches' wave priority
# (10 steps each, interleaved twice), then the config-4 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-prio}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -1 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
STEPS=10 bash tools/gpu_ab_trees.sh ${1:-prio} "prio|.|" "noprio|.|MANDO_LIB=abl/noprio/libmando.so" || exit 1
if [ -n "$C4" ]; then
  timeout -k 10 900 python3 bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > $D/bench_config4.json 2> $D/bench_config4.err || { echo "config4 failed"; tail -5 $D/bench_config4.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_config4.json')); print('config4', d['value'], round(d['ms_per_step'], 1), d['config']['phases_rank0_s'])"
fi
