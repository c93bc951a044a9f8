# GPU box: stale-bytes probe, per-phase POA cycles (MANDO_PROF=1) on config-3-shaped groups, and the
# config-3 stage timeline.  usage: RUN=r03b bash tools/gpu_prof3.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-p3}
mkdir -p $D
export TMPDIR=/tmp
if [ -z "$SKIP_PROBE" ]; then
  timeout -k 10 240 ./tools/stale_probe > $D/stale_probe.txt 2>&1 || { echo "probe failed"; cat $D/stale_probe.txt; exit 1; }
  cat $D/stale_probe.txt
fi
MANDO_PROF=1 timeout -k 10 300 python tools/prof.py ${NG:-4000} > $D/prof3.txt 2>&1 || { echo "prof failed"; tail -20 $D/prof3.txt; exit 1; }
grep -E "mando prof|groups" $D/prof3.txt | cut -c1-300
timeout -k 10 300 python tools/e2e_timeline.py 20000 > $D/timeline.txt 2>&1 && tail -14 $D/timeline.txt
