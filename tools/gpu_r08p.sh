# Update pass 1 split (batched lookups, then edges): POA byte-exactness, then the phase split on
# config-4-shaped groups (default build and the -DMANDO_UPD_PROF dev build of the same sources).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08p}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py tests/test_define_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $D/pytest.log | head -30 | cut -c1-300; exit $rc; }
P="LEN_LO=2000 LEN_HI=3600 DEPTH=25"
env MANDO_PROF=1 $P timeout -k 10 300 python3 tools/prof.py 20000 > $D/prof_default.txt 2>&1 || { echo "prof failed"; tail -5 $D/prof_default.txt; exit 1; }
env MANDO_PROF=1 $P MANDO_LIB=variants/updprof2/libmando.so timeout -k 10 300 python3 tools/prof.py 20000 > $D/prof_updprof.txt 2>&1 || { echo "updprof failed"; tail -5 $D/prof_updprof.txt; exit 1; }
grep -h "cycles per read\|per DP row\|groups" $D/prof_*.txt
