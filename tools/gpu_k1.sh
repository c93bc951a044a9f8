# GPU box: clustering parity (cluster + define tests), config-2 bench with clustering stage times,
# and the K1/K2 phase cycles of a MANDO_CL_PHASES build (build/clph).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${RUN:-k1}; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_cluster_gpu.py tests/test_cluster.py tests/test_define_ref.py tests/test_define_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; grep -E "passed|failed" $D/pytest.log | tail -2 | cut -c1-200
[ $rc -eq 0 ] || { tail -40 $D/pytest.log | cut -c1-300; exit $rc; }
MANDO_CL_TIME=1 timeout -k 10 400 python bench.py --workload config2 --steps 2 --warmup 1 --no-cpu-baseline > $D/c2.json 2> $D/c2.err || { tail -20 $D/c2.err; exit 1; }
cut -c1-400 $D/c2.json; grep -h "\[cluster\]" $D/c2.err | tail -4
MANDO_LIB=build/clph/libmando.so timeout -k 10 400 python bench.py --workload config2 --steps 1 --warmup 0 --no-cpu-baseline > $D/c2ph.json 2> $D/c2ph.err || { tail -20 $D/c2ph.err; exit 1; }
grep -h -E "phases|peaks" $D/c2ph.err | head -30
timeout -k 10 300 python tools/prof.py 4000 > $D/prof3.txt 2>&1 || { tail -5 $D/prof3.txt; exit 1; }
grep -h -E "mando prof|groups" $D/prof3.txt | cut -c1-220
MANDO_CL_TIME=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/c3.json 2> $D/c3.err || { tail -20 $D/c3.err; exit 1; }
cut -c1-300 $D/c3.json; grep -h "\[cluster\]" $D/c3.err | tail -4
