set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/def; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_define_gpu.py tests/test_define_ref.py tests/test_cluster.py -x -q -m gpu --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -1 $D/pytest.log | cut -c1-200
[ $rc -eq 0 ] || { tail -40 $D/pytest.log | cut -c1-300; exit $rc; }
VARIANTS="X=0" bash tools/gpu_chunks.sh 2>&1 | grep -v "^\[cluster\]"
