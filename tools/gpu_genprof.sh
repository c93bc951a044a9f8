set -o pipefail
cd $GRAFT_REPO_ROOT
for L in "7000 8000"; do
  set -- $L
  MANDO_LIB=build/genprof/libmando.so DEPTH=${DEPTH:-60} LEN_LO=$1 LEN_HI=$2 timeout -k 10 300 python tools/prof.py ${N:-16} 2>&1 | grep -E "fast rows|cycles per read|seg0|groups" | cut -c1-200
done
