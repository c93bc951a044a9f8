# POA fast rows with buffer-descriptor stores: parity first, then an interleaved A/B against the
# previous build (abv/base) on the config-3 and config-4 group shapes (tools/prof.py, MANDO_PROF).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08w}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_poa_gpu.py tests/test_abpoa_cli.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest_poa.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_poa.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $D/pytest_poa.log | head -20 | cut -c1-300; exit $rc; }
run() {
  MANDO_LIB=$2 timeout -k 10 200 python tools/prof.py ${NG:-20000} > $D/$1.log 2>&1 || { echo "$1 failed"; tail -3 $D/$1.log; return 1; }
  echo "$1: $(grep -o 'dp [0-9]* ([0-9.]*/row)' $D/$1.log) $(grep -o 'backtrack [0-9]*' $D/$1.log | head -1) $(grep -o 'kernel [0-9.]* ms' $D/$1.log)"
}
for pass in 1 2; do
  run c3_base.$pass abv/base/libmando.so || exit 1
  run c3_new.$pass mandalorion_amd/lib/libmando.so || exit 1
done
export LEN_LO=2000 LEN_HI=3600 DEPTH=25
for pass in 1 2; do
  run c4_base.$pass abv/base/libmando.so || exit 1
  run c4_new.$pass mandalorion_amd/lib/libmando.so || exit 1
done
