# POA fast rows with the rare reload / mask blocks out of line (one taken branch per chain row instead
# of three): parity, then an interleaved A/B against abv/base on the config-3 and config-4 shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08y}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_poa_gpu.py tests/test_abpoa_cli.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest_poa.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_poa.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $D/pytest_poa.log | head -20 | cut -c1-300; exit $rc; }
run() {
  MANDO_LIB=$2 timeout -k 10 200 python tools/prof.py ${NG:-20000} > $D/$1.log 2>&1 || { echo "$1 failed"; tail -3 $D/$1.log; return 1; }
  echo "$1: $(grep -o 'dp [0-9]* ([0-9.]*/row)' $D/$1.log) $(grep -o 'kernel [0-9.]* ms' $D/$1.log)"
}
for shape in c3 c4; do
  if [ $shape = c4 ]; then export LEN_LO=2000 LEN_HI=3600 DEPTH=25; fi
  for pass in 1 2 3; do
    run $shape.base.$pass abv/base/libmando.so || exit 1
    run $shape.new.$pass mandalorion_amd/lib/libmando.so || exit 1
  done
done
