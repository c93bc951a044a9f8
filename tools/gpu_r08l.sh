# POA phase split on config-4-shaped groups: default build, the update passes (-DMANDO_UPD_PROF) and the
# backtrack's run statistics (-DMANDO_BT_STATS), dev builds under variants/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08l}
mkdir -p $D
P="LEN_LO=2000 LEN_HI=3600 DEPTH=25"
env MANDO_PROF=1 $P timeout -k 10 300 python3 tools/prof.py 20000 > $D/prof_default.txt 2>&1 || { echo "prof failed"; tail -5 $D/prof_default.txt; exit 1; }
env MANDO_PROF=1 $P MANDO_LIB=variants/updprof/libmando.so timeout -k 10 300 python3 tools/prof.py 20000 > $D/prof_updprof.txt 2>&1 || { echo "updprof failed"; tail -5 $D/prof_updprof.txt; exit 1; }
env MANDO_PROF=1 MANDO_BT_STATS=1 $P MANDO_LIB=variants/btstats/libmando.so timeout -k 10 300 python3 tools/prof.py 20000 > $D/prof_btstats.txt 2>&1 || { echo "btstats failed"; tail -5 $D/prof_btstats.txt; exit 1; }
grep -h "mando prof\|groups" $D/prof_*.txt
