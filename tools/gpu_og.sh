set -o pipefail
cd $GRAFT_REPO_ROOT
VARIANTS="${VARIANTS:-MANDO_STREAM_PRIO=0 X=0 MANDO_FIRST_CHUNK=0.2}" bash tools/gpu_chunks.sh
