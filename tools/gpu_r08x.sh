# Interleaved A/B of fast-row variants (tools/prof.py, MANDO_PROF): base, head-only (vA), stores-only
# (vB), both (in-tree), on the config-3 and config-4 group shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08x}
mkdir -p $D
run() {
  MANDO_LIB=$2 timeout -k 10 200 python tools/prof.py ${NG:-20000} > $D/$1.log 2>&1 || { echo "$1 failed"; tail -3 $D/$1.log; return 1; }
  echo "$1: $(grep -o 'dp [0-9]* ([0-9.]*/row)' $D/$1.log) $(grep -o 'kernel [0-9.]* ms' $D/$1.log)"
}
for shape in c3 c4; do
  if [ $shape = c4 ]; then export LEN_LO=2000 LEN_HI=3600 DEPTH=25; fi
  for pass in 1 2; do
    for v in base vA vB new; do
      lib=abv/$v/libmando.so; [ $v = new ] && lib=mandalorion_amd/lib/libmando.so
      run $shape.$v.$pass $lib || exit 1
    done
  done
done
