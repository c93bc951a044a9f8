set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/cl2; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_cluster_gpu.py tests/test_cluster.py -x -q -m gpu --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -2 $D/pytest.log | cut -c1-200
[ $rc -eq 0 ] || { tail -30 $D/pytest.log | cut -c1-300; exit $rc; }
LIBV=MANDO_LIB=build/clph/libmando.so bash tools/gpu_c2.sh 2>&1 | grep -E "phases|cluster\]" | head -12
VARIANTS="X=0" bash tools/gpu_chunks.sh 2>&1 | tail -5
