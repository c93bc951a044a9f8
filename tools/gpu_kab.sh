# GPU box: parity of the in-tree libmando (POA and D-driver GPU tests), then the POA kernel A/B over
# several builds (tools/ab_prof.sh, config-3-shaped groups) and optional extras.
# usage: bash tools/gpu_kab.sh TAG name=path/to/libmando.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-kab}; shift
D=gpurun_out/$T
mkdir -p $D
if [ -n "$UBENCH" ]; then timeout -k 10 120 ./tools/ubench_issue > $D/ubench.txt 2>&1 && cat $D/ubench.txt || exit 1; fi
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_poa_gpu.py tests/test_define_ref.py tests/test_abpoa_cli.py} -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
  rc=$?; tail -3 $D/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $D/pytest.log | head -20; exit $rc; }
fi
if [ -n "$ROWSTATS" ]; then MANDO_LIB=$ROWSTATS timeout -k 10 200 python3 tools/prof.py 4000 > $D/rowstats.txt 2>&1 && grep "prof\]" $D/rowstats.txt | cut -c1-250 || exit 1; fi
bash tools/ab_prof.sh $T "$@"
