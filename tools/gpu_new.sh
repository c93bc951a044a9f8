# GPU box: the new reference-pinned / config tests, then the config-2 and config-5 D-module benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/${RUN:-new}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_define_ref.py tests/test_abpoa_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $D/pytest.log
[ $rc -eq 0 ] || exit $rc
for w in config2 config5; do
  timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $D/bench_$w.json 2> $D/bench_$w.err || { echo "bench $w failed"; tail -5 $D/bench_$w.err; exit 1; }
  cat $D/bench_$w.json
done
