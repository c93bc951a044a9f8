# GPU box: parity of the in-tree libmando (POA + D-driver GPU tests), the POA phase profile of config-5-shaped
# unseeded groups (tools/prof.py), then the config-4 bench line (10M records, N=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-c4c5}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py tests/test_define_ref.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -2 $D/pytest.log; [ $rc -eq 0 ] || exit $rc
DEPTH=100 LEN_LO=8300 LEN_HI=8700 timeout -k 10 300 python3 tools/prof.py 16 > $D/prof_c5.txt 2>&1 && grep "prof\]\|groups" $D/prof_c5.txt | cut -c1-260 || exit 1
timeout -k 10 900 python3 bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > $D/bench_config4.json 2> $D/bench_config4.err
rc=$?; tail -3 $D/bench_config4.err; cat $D/bench_config4.json; exit $rc
