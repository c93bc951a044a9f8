# GPU box: POA tests, then config 5 with -S team sizes 1 / auto and the previous build.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-team}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $D/pytest.log | tail -5 | cut -c1-300
[ $rc -eq 0 ] || { tail -40 $D/pytest.log | cut -c1-300; exit $rc; }
for v in "MANDO_TEAM=1" "MANDO_X=0" "MANDO_LIB=build/head/libmando.so"; do
  env $v MANDO_PROF=1 timeout -k 10 400 python bench.py --workload config5 --steps 1 --warmup 1 --no-cpu-baseline > $D/c5.json 2> $D/c5.err || { echo "$v failed"; tail -20 $D/c5.err; exit 1; }
  echo "== $v"; grep -E "team|cycles per read|Gcycles" $D/c5.err | tail -8 | cut -c1-200
  python3 -c "import json,sys; d=json.load(open('$D/c5.json')); print(d['ms_per_step'], d['config']['phases_rank0_s'], d['config']['poa_kernel']['kernel_ms_total'])"
done
