# GPU box: config-3 stage timelines (tools/e2e_timeline.py) with the async POA pipeline on and off,
# each POA launch logged (MANDO_LAUNCH_LOG: lane, slots, waves per CU, grid; per-kind launch intervals).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-tl}
mkdir -p $D
export TMPDIR=/tmp
for a in ${MODES:-1 0}; do
  MANDO_LAUNCH_LOG=1 MANDO_POA_ASYNC=$a timeout -k 10 300 python3 tools/e2e_timeline.py > $D/timeline_async$a.txt 2>&1 || { tail -5 $D/timeline_async$a.txt; exit 1; }
done
grep -h "total\|poa launch\|poa \|orient\|cluster \|mando launch" $D/timeline_async*.txt
