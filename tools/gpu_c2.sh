set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c2
env ${LIBV:-} MANDO_CL_TIME=1 timeout -k 10 400 python bench.py --workload config2 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/c2/out.txt 2> gpurun_out/c2/err.txt || { tail -20 gpurun_out/c2/err.txt; exit 1; }
grep -h -E "\[cluster\]|phases" gpurun_out/c2/err.txt gpurun_out/c2/out.txt | head -40
