# DP cycles per row against resident waves per SIMD (MANDO_WAVES_PER_CU = 4 / 8 / 12 / 16 one-wave
# workgroups per CU), tools/prof.py on the config-3 and config-4 group shapes at HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08ac}
mkdir -p $D
for shape in c3 c4; do
  if [ $shape = c4 ]; then export LEN_LO=2000 LEN_HI=3600 DEPTH=25; fi
  for w in 4 8 12 16; do
    MANDO_WAVES_PER_CU=$w timeout -k 10 300 python tools/prof.py 20000 > $D/$shape.w$w.log 2>&1 || { echo "$shape w$w failed"; tail -3 $D/$shape.w$w.log; exit 1; }
    echo "$shape waves/CU $w: $(grep -o 'desc [0-9]*' $D/$shape.w$w.log) $(grep -o 'dp [0-9]* ([0-9.]*/row)' $D/$shape.w$w.log) $(grep -o 'backtrack [0-9]*' $D/$shape.w$w.log | head -1) $(grep -o 'update [0-9]*' $D/$shape.w$w.log) $(grep -o 'kernel [0-9.]* ms' $D/$shape.w$w.log)"
  done
done
