# GPU box: orientation parity tests with the current build, then orient_bench2 A/B (MANDO_LIB) twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-oab}
mkdir -p $D
A=${A:-build/oold/libmando.so}; B=${B:-mandalorion_amd/lib/libmando.so}
timeout -k 10 120 python -u -m pytest tests/test_orient.py -m gpu -x -v --timeout 60 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; grep -E "passed|failed" $D/pytest.log | tail -3; [ $rc -eq 0 ] || { tail -40 $D/pytest.log; exit $rc; }
for i in 1 2; do
  for v in A B; do
    L=$A; [ $v = B ] && L=$B
    MANDO_LIB=$L timeout -k 10 300 python tools/orient_bench2.py 20000 0.3 > $D/$v$i.log 2>&1 || { tail -5 $D/$v$i.log; exit 1; }
    echo "$v$i $(cat $D/$v$i.log)"
  done
done
if [ -f build/oprof/libmando.so ]; then
  MANDO_LIB=build/oprof/libmando.so timeout -k 10 300 python tools/orient_bench2.py 20000 0.3 > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
  tail -3 $D/prof.log
fi
