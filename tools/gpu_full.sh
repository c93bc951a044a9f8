# GPU box: every gpu test, smoke, the default bench line and the stage timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-full}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $D/pytest.log | tail -5 | cut -c1-300
[ $rc -eq 0 ] || { tail -60 $D/pytest.log | cut -c1-300; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo smoke failed; tail $D/smoke.log; exit 1; }
cat $D/smoke.log
timeout -k 10 500 python bench.py ${BARGS:-} > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
timeout -k 10 300 python tools/e2e_timeline.py 20000 > $D/timeline.txt 2>&1 && tail -12 $D/timeline.txt
