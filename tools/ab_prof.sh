# Dev A/B on the GPU box: tools/prof.py (config-3 shape, 20,000 groups) with several libmando builds,
# interleaved twice.  usage: bash tools/ab_prof.sh TAG name=path/to/libmando.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-ab}
shift
mkdir -p $D
run() {
  MANDO_LIB=$2 timeout -k 10 200 python tools/prof.py ${NG:-20000} > $D/$1.log 2>&1 || { echo "$1 failed"; tail -3 $D/$1.log; return 1; }
  echo "$1: $(grep -o 'desc [0-9]*' $D/$1.log) $(grep -o 'dp [0-9]* ([0-9.]*/row)' $D/$1.log) $(grep -o 'backtrack [0-9]*' $D/$1.log | head -1) $(grep -o 'update [0-9]*' $D/$1.log) $(grep -o 'kernel [0-9.]* ms' $D/$1.log)"
}
for pass in 1 2; do
  for kv in "$@"; do
    run "${kv%%=*}.$pass" "${kv#*=}" || exit 1
  done
done
