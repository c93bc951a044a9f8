# GPU box: POA parity, then config-3 bench lines with and without the launch-kind stagger
# (MANDO_POA_STAGGER=1; 10 steps each, interleaved twice).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-stag}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -1 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
STEPS=10 bash tools/gpu_ab_trees.sh ${1:-stag} "stag|.|MANDO_POA_STAGGER=1" "nostag|.|"
