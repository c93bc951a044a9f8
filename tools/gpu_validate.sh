set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-val}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $D/pytest.log 2>&1
echo "pytest rc=$?"; tail -3 $D/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 && echo "smoke ok" && cat $D/smoke.log &&
timeout -k 10 500 python bench.py > $D/bench.json 2> $D/bench.err; echo "bench rc=$?"; cat $D/bench.json
