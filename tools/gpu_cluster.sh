# GPU box: clustering kernels vs the restatement, then the D-module tests that now run them.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-cl}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_cluster_gpu.py ${EXTRA:-} -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 $D/pytest.log | cut -c1-400
exit $rc
