# GPU box: lone long groups (MANDO_PROF=1 per-phase cycles), interleaved twice: the one-wave wide kernel at
# 128 VGPRs (base), at 256 VGPRs (build/wide2), and two-wave workgroups (W2=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-w2ab}
mkdir -p $D
run() {  # name lib w2 lo hi depth n
  MANDO_LIB=$2 MANDO_POA_W2=$3 LEN_LO=$4 LEN_HI=$5 DEPTH=$6 timeout -k 10 300 python3 tools/prof.py $7 > $D/$1.txt 2>&1 || { echo "$1 failed"; tail -5 $D/$1.txt; return 1; }
  echo "$1: $(grep -o 'dp [0-9]* ([0-9.]*/row)' $D/$1.txt) $(grep -o 'backtrack [0-9]*' $D/$1.txt | head -1) $(grep -o 'update [0-9]*' $D/$1.txt) $(grep -o 'consensus/slot [0-9]*' $D/$1.txt) $(grep -o 'kernel [0-9.]* ms' $D/$1.txt)"
}
for pass in 1 2; do
  for shape in "8300 8700 100 16" "5000 6000 50 64"; do
    set -- $shape
    run base_$1_$pass mandalorion_amd/lib/libmando.so 0 $1 $2 $3 $4 || exit 1
    run wide2_$1_$pass variants/wide2/libmando.so 0 $1 $2 $3 $4 || exit 1
    run w2_$1_$pass mandalorion_amd/lib/libmando.so 1 $1 $2 $3 $4 || exit 1
  done
done
