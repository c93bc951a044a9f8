# GPU box, round end: every GPU test, smoke, then the 2/4/8-rank rehearsals of configs 3 and 4 with the
# one-GPU bench lines (tools/gpu_r04n.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r04f}_tests bash tools/gpu_r04_tests.sh || exit 1
TAG=${TAG:-r04f} bash tools/gpu_r04n.sh
