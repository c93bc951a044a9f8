# GPU box: orientation parity tests, then the config-3 bench under a kernel trace (orientation kernel times)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${RUN:-olpt}; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_orient.py tests/test_define_gpu.py tests/test_define_ref.py -x -q -m gpu --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -1 $D/pytest.log; [ $rc -eq 0 ] || { tail -30 $D/pytest.log; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { tail -5 $D/bench.err; exit 1; }
cut -c1-200 $D/bench.json
grep -h "orient_kernel\|poa_kernel" $(find $D/prof -name "*kernel_stats.csv") | cut -c1-160
