# Round 6 first GPU call: GPU tests at HEAD, a config-4 trace (kernels + DMA copies + HIP API) for the
# blit / pipeline-gap analysis (tools/blit_origin.py), the concurrent page-cache reads of the 8-rank plan,
# and the default bench line (host CPU per step with per-wait blocking-sync events).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08a}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $D/pytest.log | head -30 | cut -c1-300; exit $rc; }
timeout -k 10 500 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench.json')); c=d['config']; print(round(d['ms_per_step'],1), c['steps_s'], c['steps_poa_kernel_ms'], c['host_cpu_s_per_step_rank0'], c['page_cache'])"
timeout -k 10 300 python3 tools/read_contention.py /tmp/mando_bench_config4_200000 8 2 3 > $D/read_contention_8x2.json 2> $D/read_contention_8x2.err || { echo "reads failed"; tail -5 $D/read_contention_8x2.err; exit 1; }
cat $D/read_contention_8x2.json
timeout -k 10 300 python3 tools/read_contention.py /tmp/mando_bench_config4_200000 8 16 3 > $D/read_contention_8x16.json 2> $D/read_contention_8x16.err || { echo "reads failed"; exit 1; }
cat $D/read_contention_8x16.json
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $D/trace -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 > $D/trace.out 2>&1 || { echo "trace failed"; tail -5 $D/trace.out; exit 1; }
python3 tools/blit_origin.py $D/trace 60 > $D/blit_origin.txt 2>&1; tail -40 $D/blit_origin.txt
du -sh $D/trace
find $D/trace -name "*hip_api_trace.csv" -size +20M -exec gzip {} \;
