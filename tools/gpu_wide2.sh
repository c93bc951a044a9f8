set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/w2; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $D/pytest.log | tail -3 | cut -c1-300
[ $rc -eq 0 ] || { tail -40 $D/pytest.log | cut -c1-300; exit $rc; }
bash tools/gpu_genprof.sh
A=build/prev/libmando.so bash tools/gpu_ab.sh
