# GPU box: POA tests, row costs (lone waves) and the config-5 bench after POA kernel changes.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-wide}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py ${EXTRA:-} -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $D/pytest.log | tail -5 | cut -c1-300
[ $rc -eq 0 ] || { tail -40 $D/pytest.log | cut -c1-300; exit $rc; }
N=64
run() { echo "== $1"; env $2 timeout -k 10 300 python tools/prof.py $N > $D/$1.log 2>&1 || { tail -5 $D/$1.log; exit 1; }; grep -E "fast rows|cycles per read|groups" $D/$1.log | cut -c1-220; }
run c3_r16 "DEPTH=20"
run long_def "DEPTH=10 LEN_LO=8000 LEN_HI=9000"
for w in ${WLS:-config5}; do
  timeout -k 10 400 python bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline > $D/$w.json 2> $D/$w.err || { echo "$w failed"; tail -20 $D/$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$D/$w.json')); print('$w', d['ms_per_step'], d['config']['phases_rank0_s'], d['config']['poa_kernel'])"
done
