# GPU box: POA parity of the in-tree library, then the wide-row A/B (abl/w0 vs abl/w1): DP cycles per row
# on config-5-shaped unseeded groups (tools/prof.py, lone waves), config-5 and config-3 bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-wide}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py tests/test_define_ref.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -1 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for v in w0 w1; do
    MANDO_LIB=abl/$v/libmando.so DEPTH=100 LEN_LO=8300 LEN_HI=8700 timeout -k 10 300 python3 tools/prof.py 16 > $D/prof_$v.$pass.txt 2>&1 || { echo "prof $v failed"; tail -3 $D/prof_$v.$pass.txt; exit 1; }
    echo "$v.$pass $(grep -o 'dp [0-9]* ([0-9.]*/row)' $D/prof_$v.$pass.txt) $(grep -o 'backtrack [0-9]*' $D/prof_$v.$pass.txt | head -1) $(grep -o 'kernel [0-9.]* ms' $D/prof_$v.$pass.txt)"
  done
done
for pass in 1 2; do
  for v in w0 w1; do
    MANDO_LIB=abl/$v/libmando.so timeout -k 10 300 python3 bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > $D/c5_$v.$pass.json 2> $D/c5_$v.$pass.err || { echo "c5 $v failed"; tail -3 $D/c5_$v.$pass.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/c5_$v.$pass.json')); print('c5 $v.$pass', round(d['ms_per_step'],1), d['config']['steps_s'])"
  done
done
STEPS=8 bash tools/gpu_ab_trees.sh $1 "c3w0|.|MANDO_LIB=abl/w0/libmando.so" "c3w1|.|MANDO_LIB=abl/w1/libmando.so"
