cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/occ
MANDO_PROF=1 timeout -k 10 300 python tools/e2e_timeline.py 20000 > gpurun_out/occ/t.txt 2>&1; rc=$?
grep -E "waves per CU|total" gpurun_out/occ/t.txt | sort | uniq -c | head -20; exit $rc
