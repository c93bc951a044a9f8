# GPU box: clustering GPU tests (the wave-parallel permutation), config-2 bench, then the HW-queue timelines.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-r03w}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cluster_gpu.py tests/test_cluster.py -m gpu > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python3 bench.py --workload config2 --steps 3 --warmup 1 --no-cpu-baseline > $D/bench_config2.json 2> $D/bench_config2.err || { tail -5 $D/bench_config2.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_config2.json')); c=d['config']; print('config2', round(d['ms_per_step'],1), c['steps_s'], c['phases_rank0_s'], c['full_output_equals_oracle'])"
bash tools/gpu_timeline_hwq.sh ${1:-r03w}
