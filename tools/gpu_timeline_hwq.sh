# GPU box: config-3 stage timelines with per-launch logs, at 4 (HIP's default) and 8 hardware queues per
# process: do the POA lanes of one batch run side by side or one after the other?
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-hwq}
mkdir -p $D
export TMPDIR=/tmp
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q MANDO_LAUNCH_LOG=1 timeout -k 10 300 python3 tools/e2e_timeline.py > $D/timeline_q$q.txt 2>&1 || { tail -5 $D/timeline_q$q.txt; exit 1; }
  echo "== GPU_MAX_HW_QUEUES=$q"
  grep -h "total\|poa \|orient\|cluster \|batch" $D/timeline_q$q.txt
done
