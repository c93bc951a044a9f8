# GPU box: backtrack-window prefetch A/B (MANDO_BT_PREFETCH) against the tree before the refactor (orig)
# and the refactored default (cur): POA GPU tests with the prefetch build, then tools/ab_prof.sh on
# config-3-shaped groups and on 8-9 kb groups (wide launches), interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04bt}
mkdir -p $D
MANDO_LIB=variants/pf/libmando.so timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_pf.log 2>&1 || { echo "pf tests failed"; tail -30 $D/pytest_pf.log; exit 1; }
tail -1 $D/pytest_pf.log
bash tools/ab_prof.sh ${TAG:-r04bt}/c3 orig=variants/orig/libmando.so cur=mandalorion_amd/lib/libmando.so pf=variants/pf/libmando.so || exit 1
NG=64 LEN_LO=8000 LEN_HI=9000 DEPTH=50 bash tools/ab_prof.sh ${TAG:-r04bt}/long orig=variants/orig/libmando.so cur=mandalorion_amd/lib/libmando.so pf=variants/pf/libmando.so
