# GPU tests, the default bench line (host CPU per step), config 5 against the reference's own clustering,
# and the POA phase profile on config-4-shaped narrow groups.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08b}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $D/pytest.log | head -30 | cut -c1-300; exit $rc; }
timeout -k 10 500 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench.json')); c=d['config']; print(round(d['ms_per_step'],1), c['steps_s'], c['steps_poa_kernel_ms'], c['host_cpu_s_per_step_rank0'], c['page_cache']['before']['resident_frac'])"
timeout -k 10 300 python3 bench.py --workload config5 --no-cpu-baseline > $D/bench_config5.json 2> $D/bench_config5.err || { echo "c5 failed"; tail -20 $D/bench_config5.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_config5.json')); c=d['config']; print('config5', round(d['ms_per_step'],1), c['clustering_equals_reference'], c['full_output_equals_oracle'])"
MANDO_PROF=1 LEN_LO=2000 LEN_HI=3600 DEPTH=25 timeout -k 10 300 python3 tools/prof.py 20000 > $D/prof_c4shape.txt 2>&1 || { echo "prof failed"; tail -5 $D/prof_c4shape.txt; exit 1; }
cat $D/prof_c4shape.txt
