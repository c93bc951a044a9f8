# GPU box: first-attempt predecessor-byte / spill capacities (MANDO_KPC_FRAC, MANDO_SVC_FRAC) on config 3:
# groups re-run, slot size, POA time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-caps}
mkdir -p $D
for v in "1.5 1.5" "0.75 1.5" "1.5 0.25" "1.5 0.5" "1.0 0.75" "0.75 0.5"; do
  set -- $v
  MANDO_KPC_FRAC=$1 MANDO_SVC_FRAC=$2 MANDO_WS_LOG=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 > $D/c3_$1_$2.json 2> $D/c3_$1_$2.err || { echo "$v failed"; tail -3 $D/c3_$1_$2.err; exit 1; }
  echo "kp $1 sv $2: $(python3 -c "import json; d=json.load(open('$D/c3_$1_$2.json')); print(d['config']['steps_poa_kernel_ms'])") $(grep -m1 're-run' $D/c3_$1_$2.err | cut -c1-90) | $(grep -m2 'slot workspace' $D/c3_$1_$2.err | tail -1 | cut -c1-60)"
done
