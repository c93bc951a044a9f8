# Dev loop on the GPU box: POA parity tests, then the phase profile (and optionally the BT-stats build).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-it}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py tests/test_define_gpu.py -x -q --timeout 240 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/prof.py ${NG:-20000} > $D/prof.log 2>&1 && cat $D/prof.log || exit 1
if [ -n "$BT" ]; then MANDO_BT_STATS=1 MANDO_LIB=build/btstats/libmando.so timeout -k 10 200 python tools/prof.py 4000 > $D/bt.log 2>&1 && cat $D/bt.log; fi
