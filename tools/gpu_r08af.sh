# Wave priorities in the POA kernel, interleaved A/B (tools/prof.py, MANDO_PROF): base (DP 0, serial 1),
# vP2 (row head at 2, serial 1), vP3 = in-tree (row head at 2, serial 3), vP4 (vP3 + scans at 2), vP5 (vP3 with
# the head window through the ring-read wait); parity first.  VARIANTS overrides the list.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08af}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_poa_gpu.py tests/test_abpoa_cli.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest_poa.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_poa.log | cut -c1-300
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $D/pytest_poa.log | head -20 | cut -c1-300; exit $rc; }
run() {
  MANDO_LIB=$2 timeout -k 10 200 python tools/prof.py ${NG:-20000} > $D/$1.log 2>&1 || { echo "$1 failed"; tail -3 $D/$1.log; return 1; }
  echo "$1: $(grep -o 'desc [0-9]*' $D/$1.log | head -1) $(grep -o 'dp [0-9]* ([0-9.]*/row)' $D/$1.log) $(grep -o 'backtrack [0-9]*' $D/$1.log | head -1) $(grep -o 'update [0-9]*' $D/$1.log | head -1) $(grep -o 'kernel [0-9.]* ms' $D/$1.log)"
}
for shape in c3 c4; do
  if [ $shape = c4 ]; then export LEN_LO=2000 LEN_HI=3600 DEPTH=25; fi
  for pass in ${PASSES:-1 2 3}; do
    for v in ${VARIANTS:-base vP2 vP3}; do
      lib=abv/$v/libmando.so; [ $v = vP3 ] && lib=mandalorion_amd/lib/libmando.so
      run $shape.$v.$pass $lib || exit 1
    done
  done
done
