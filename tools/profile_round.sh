set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r01c
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --e2e-loci 0 > gpurun_out/r01c/bench.json 2> gpurun_out/r01c/bench.err
echo "bench rc=$?"
cat gpurun_out/r01c/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r01c/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --e2e-loci 0 > gpurun_out/r01c/prof.out 2>&1
echo "prof rc=$?"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r01c/pmcf -o f --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --e2e-loci 0 > gpurun_out/r01c/pmcf.out 2>&1
echo "pmcf rc=$?"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r01c/pmcw -o w --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --e2e-loci 0 > gpurun_out/r01c/pmcw.out 2>&1
echo "pmcw rc=$?"
find gpurun_out/r01c -name "*.csv" | head -20
