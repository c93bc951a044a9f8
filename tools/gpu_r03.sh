# Round-3 GPU session: box facts, the stale-bytes probe, every GPU test, smoke, bench lines (config 3
# default, configs 2 and 5 with their full-size output checks).  usage: RUN=r03a bash tools/gpu_r03.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-r03}
mkdir -p $D
export TMPDIR=/tmp
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; df -h /tmp | tail -1; free -g | head -2; } > $D/box.txt 2>&1; cat $D/box.txt
if [ -z "$SKIP_PROBE" ]; then
  timeout -k 10 180 ./tools/stale_probe > $D/stale_probe.txt 2>&1 || { echo "probe failed"; cat $D/stale_probe.txt; exit 1; }
  cat $D/stale_probe.txt
fi
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|SKIPPED" $D/pytest.log | tail -8 | cut -c1-300
  [ $rc -eq 0 ] || { tail -60 $D/pytest.log | cut -c1-300; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo smoke failed; tail $D/smoke.log; exit 1; }
  cat $D/smoke.log
fi
timeout -k 10 600 python bench.py ${BARGS:-} > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench.json')); print('config3', d['value'], d['ms_per_step'], d['config']['steps_s'], d['config']['steps_poa_kernel_ms'], d['config']['full_output_equals_oracle'], d['roofline']['frac'], d.get('cpu_baseline'))"
for w in ${WLS:-config2 config5}; do
  timeout -k 10 500 python bench.py --workload $w --no-cpu-baseline > $D/bench_$w.json 2> $D/bench_$w.err || { echo "$w failed"; tail -20 $D/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$w.json')); print('$w', round(d['ms_per_step'], 1), d['config']['phases_rank0_s'], d['config']['full_output_equals_oracle'])"
done
