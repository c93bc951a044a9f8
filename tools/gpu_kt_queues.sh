# GPU box: kernel trace of the config-3 stage timeline (two D passes), kernels listed with their HW queue
# and stream for the last pass.  usage: Q=4 bash tools/gpu_kt_queues.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-ktq}
mkdir -p $D
export TMPDIR=/tmp
env ${Q:+GPU_MAX_HW_QUEUES=$Q} MANDO_WS_LOG=1 timeout -k 10 400 rocprofv3 --kernel-trace -d $D/kt -o kt --output-format csv -- python3 tools/e2e_timeline.py > $D/timeline.txt 2>&1 || { tail -20 $D/timeline.txt; exit 1; }
F=$(find $D/kt -name "*kernel_trace.csv" | head -1)
python3 tools/kt_queues.py $F --last-ms ${LAST:-2600} > $D/queues.txt
grep -h "total\|poa \|orient\|cluster \|batch" $D/timeline.txt
cat $D/queues.txt | head -120
