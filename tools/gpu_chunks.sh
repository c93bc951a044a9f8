# GPU box: config-3 D-module timelines under pipeline variants (chunk fractions, POA waves per CU).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-ch}; mkdir -p $D
export TMPDIR=/tmp
i=0
for v in ${VARIANTS:-"X=0"}; do
  i=$((i+1))
  env $v MANDO_CL_TIME=1 timeout -k 10 300 python tools/e2e_timeline.py 20000 > $D/t$i.txt 2>&1 || { echo "$v failed"; tail $D/t$i.txt; exit 1; }
  echo "== $v: $(grep 'total' $D/t$i.txt | head -1)"; grep -E "^  (cluster|orient|poa|write) " $D/t$i.txt | tr '\n' ' ' | cut -c1-600; echo; grep "^\[cluster\]" $D/t$i.txt | tail -2
done
