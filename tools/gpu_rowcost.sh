# GPU box: DP cycles per row by row kind (MANDO_PROF=1, tools/prof.py), lone waves (few groups).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-rc}
mkdir -p $D
N=${N:-64}
run() { echo "== $1"; env $2 timeout -k 10 300 python tools/prof.py $N > $D/$1.log 2>&1 || { tail -5 $D/$1.log; exit 1; }; grep -E "fast rows|cycles per read|groups" $D/$1.log | cut -c1-220; }
run c3_r16 "DEPTH=20"
run c3_r32fast "DEPTH=20 MANDO_POA_DBG=1"
run c3_r32gen "DEPTH=20 MANDO_POA_DBG=5"
run c3_r16gen "DEPTH=20 MANDO_POA_DBG=2"
run long_def "DEPTH=10 LEN_LO=8000 LEN_HI=9000"
