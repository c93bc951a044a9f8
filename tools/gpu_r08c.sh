# GPU tests (fused gather + encode), the default bench line (cpu_baseline = the SIMD restatement), the
# RCCL exchange beside a POA grid, and the SQC counters this device offers.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08c}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $D/pytest.log | head -30 | cut -c1-300; exit $rc; }
timeout -k 10 600 python3 bench.py > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench.json')); c=d['config']; print(round(d['value']), round(d['ms_per_step'],1), c['steps_s'], c['steps_poa_kernel_ms'], c['host_cpu_s_per_step_rank0'], d['cpu_baseline'])"
timeout -k 10 300 python3 tools/rccl_beside_poa.py 32 20000 > $D/rccl_beside_poa.json 2> $D/rccl_beside_poa.err || { echo "rccl failed"; tail -20 $D/rccl_beside_poa.err; exit 1; }
cat $D/rccl_beside_poa.json
timeout -k 10 60 rocprofv3 -L > $D/counters.txt 2>&1; grep -i -E "SQC|IFETCH|INST_CACHE|ICACHE" $D/counters.txt | head -40
timeout -k 10 300 python3 tools/bench_p.py 100000 16 --gpu > $D/bench_p.json 2> $D/bench_p.err || { echo "bench_p failed"; tail -20 $D/bench_p.err; exit 1; }
cat $D/bench_p.json
