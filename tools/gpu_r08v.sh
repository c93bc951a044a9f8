# Final check at HEAD: every GPU test, smoke, the default bench line (CPU baseline included).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08v}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $D/pytest.log | head -30 | cut -c1-300; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo smoke failed; tail $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 600 python3 bench.py > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench.json')); c=d['config']; print(round(d['value']), round(d['ms_per_step'],1), c['steps_s'], d['roofline']['frac'], d['roofline']['traffic_source'], d['cpu_baseline']['value'], c['clustering_equals_reference'], c['full_output_equals_oracle'])"
