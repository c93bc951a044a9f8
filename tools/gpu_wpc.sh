# GPU box: POA tests, then config-3 D-module totals under MANDO_WAVES_PER_CU caps (occupancy sensitivity).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-wpc}; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for v in ${VARIANTS:-X=0 MANDO_WAVES_PER_CU=14 MANDO_WAVES_PER_CU=12 X=1}; do
  env $v timeout -k 10 300 python tools/e2e_timeline.py 20000 > $D/$v.txt 2>&1 || { echo "$v failed"; tail $D/$v.txt; exit 1; }
  echo "== $v: $(grep "== chunks" $D/$v.txt | head -1)"
  grep -E "^  poa " $D/$v.txt | tr '\n' ' '; echo
done
