set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2ep
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/e2ep/prof -o run -- python3 -u $GRAFT_REPO_ROOT/tools/e2e_timeline.py 20000 > $GRAFT_REPO_ROOT/gpurun_out/e2ep/e2e.log 2>&1
echo rc=$?
tail -25 $GRAFT_REPO_ROOT/gpurun_out/e2ep/e2e.log
find $GRAFT_REPO_ROOT/gpurun_out/e2ep/prof -name "*stats.csv" | head
