set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -x -q --timeout 300 --timeout-method thread -k "grid_modes" 2>&1 | tail -2
VARIANTS="${VARIANTS:-X=0 MANDO_FIRST_CHUNK=0.15 MANDO_FIRST_CHUNK=0.2 MANDO_POA_STREAMS=1}" bash tools/gpu_chunks.sh
