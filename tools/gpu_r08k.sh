# GPU tests and smoke with every library stream on its own hardware queue; the RCCL exchange beside a
# POA grid again (r08c ran it with HIP's shared queues).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08k}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $D/pytest.log | head -30 | cut -c1-300; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo smoke failed; tail $D/smoke.log; exit 1; }
tail -2 $D/smoke.log
timeout -k 10 300 python3 tools/rccl_beside_poa.py 32 20000 > $D/rccl_beside_poa.json 2> $D/rccl.err || { echo "rccl failed"; tail -20 $D/rccl.err; exit 1; }
tail -1 $D/rccl_beside_poa.json
