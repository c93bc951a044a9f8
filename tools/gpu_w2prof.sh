# GPU box: per-phase POA cycles (MANDO_PROF=1) of lone long groups, one vs two waves per group.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-w2prof}
mkdir -p $D
for shape in "8300 8700 100 16" "5000 6000 50 16"; do
  set -- $shape
  for w2 in 0 1; do
    MANDO_POA_W2=$w2 LEN_LO=$1 LEN_HI=$2 DEPTH=$3 timeout -k 10 300 python3 tools/prof.py $4 > $D/prof_${1}_w$w2.txt 2>&1 || { echo "prof $shape w2=$w2 failed"; tail -5 $D/prof_${1}_w$w2.txt; exit 1; }
    echo "== len $1-$2 depth $3 w2=$w2"; grep -E "cycles per read|groups" $D/prof_${1}_w$w2.txt | cut -c1-220
  done
done
