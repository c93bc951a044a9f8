# GPU box: sliced root-size scan -- the multi-rank GPU tests, then the config-4 rehearsals (tools/gpu_r04n.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04rs}
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_define_ref.py tests/test_split.py > $D/pytest.log 2>&1 || { tail -20 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
WS=config4 TAG=${TAG:-r04rs} bash tools/gpu_r04n.sh
