# GPU tests (SAM and split GPU paths among them), module P timings (GPU vs host), smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08f}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $D/pytest.log | head -30 | cut -c1-300; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo smoke failed; tail $D/smoke.log; exit 1; }
tail -2 $D/smoke.log
timeout -k 10 300 python3 tools/bench_p.py 100000 16 --gpu > $D/bench_p.json 2> $D/bench_p.err || { echo "bench_p failed"; tail -20 $D/bench_p.err; exit 1; }
cat $D/bench_p.json
