# GPU box, round-3 end: every GPU test and smoke; the PMC HBM passes (FETCH_SIZE, WRITE_SIZE; separate runs)
# of one config-3 step; the default bench line reading that traffic; a rocprofv3 kernel-trace summary of
# the same command; one SQ pass; a 20-step bench (step-time spread); the stage timeline; configs 2 and 5.
# usage: TAG=r03f MANDO_COMMIT=<sha> bash tools/gpu_r03_end.sh   (outputs under gpurun_out/$TAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r03end}
D=gpurun_out/$T
mkdir -p $D
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; } > $D/box.txt 2>&1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $D/pytest.log | tail -2 | cut -c1-200
  [ $rc -eq 0 ] || { grep -E "FAILED|Error" $D/pytest.log | head -20 | cut -c1-300; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo smoke failed; tail $D/smoke.log; exit 1; }
  cat $D/smoke.log
fi
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $D/pmcf -o f --output-format csv -- $B --steps 1 --warmup 0 > $D/pmcf.out 2>&1 || { echo "pmcf failed"; tail -5 $D/pmcf.out; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $D/pmcw -o w --output-format csv -- $B --steps 1 --warmup 0 > $D/pmcw.out 2>&1 || { echo "pmcw failed"; tail -5 $D/pmcw.out; exit 1; }
F=$(find $D/pmcf -name "*counter_collection.csv" | head -1); W=$(find $D/pmcw -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py $F $W config3:20000 $D/pmc_latest.json || exit 1
timeout -k 10 500 python3 bench.py --pmc-json $D/pmc_latest.json > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -5 $D/bench.err; exit 1; }
cat $D/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- $B --steps 3 --warmup 1 --pmc-json $D/pmc_latest.json > $D/prof.out 2>&1 || { echo "prof failed"; tail -5 $D/prof.out; exit 1; }
tail -1 $D/prof.out | cut -c1-400
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $D/pmcsq -o s --output-format csv -- $B --steps 1 --warmup 0 > $D/pmcsq.out 2>&1 || { echo "sq pass failed"; tail -5 $D/pmcsq.out; exit 1; }
python3 tools/pmc_sq.py $(find $D/pmcsq -name "*counter_collection.csv" | head -1) > $D/sq.txt && head -3 $D/sq.txt | cut -c1-300
timeout -k 10 400 $B --steps 20 --warmup 1 --pmc-json $D/pmc_latest.json > $D/bench20.json 2> $D/bench20.err || { echo "bench20 failed"; tail -5 $D/bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench20.json')); s=d['config']['steps_s']; import statistics as st; m=st.median(s); print('20 steps: median', m, 'max', max(s), 'max/median', round(max(s)/m, 3), 'value', d['value'])"
timeout -k 10 300 python3 tools/e2e_timeline.py 20000 > $D/timeline.txt 2>&1 && tail -14 $D/timeline.txt
for w in config2 config5; do
  timeout -k 10 400 $B --workload $w > $D/bench_$w.json 2> $D/bench_$w.err || { echo "$w failed"; tail -5 $D/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$w.json')); print('$w', round(d['ms_per_step'], 1), d['config']['phases_rank0_s'], d['config'].get('full_output_equals_oracle'))"
done
if [ -n "$C4" ]; then
  timeout -k 10 900 $B --workload config4 --steps 1 --warmup 1 > $D/bench_config4.json 2> $D/bench_config4.err || { echo "config4 failed"; tail -5 $D/bench_config4.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_config4.json')); print('config4', d['value'], round(d['ms_per_step'], 1), d['config']['phases_rank0_s'])"
fi
