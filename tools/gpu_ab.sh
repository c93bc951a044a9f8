# GPU box: A/B of two libmando builds (MANDO_LIB) on POA row cost (lone waves) and full-chip kernel time.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-ab}
mkdir -p $D
A=${A:-build/head/libmando.so}; B=${B:-mandalorion_amd/lib/libmando.so}
run() { env $3 MANDO_LIB=$2 timeout -k 10 300 python tools/$4 > $D/$1.log 2>&1 || { tail -5 $D/$1.log; exit 1; }; echo "$1 $(grep -E 'cycles per read' $D/$1.log | sed 's/.*dp [0-9]* (\([0-9.]*\)\/row).*/\1 cyc\/row/' | tr '\n' ' ') $(grep -E '^groups' $D/$1.log)"; }
for i in 1 2; do
  run lone_A$i $A "DEPTH=20" "prof.py 64"
  run lone_B$i $B "DEPTH=20" "prof.py 64"
  run full_A$i $A "" "run_poa.py 4000"
  run full_B$i $B "" "run_poa.py 4000"
done
