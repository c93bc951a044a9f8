set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/w3; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -1 $D/pytest.log | cut -c1-200
[ $rc -eq 0 ] || { tail -40 $D/pytest.log | cut -c1-300; exit $rc; }
for L in "A=build/prev/libmando.so" "A=mandalorion_amd/lib/libmando.so"; do
  env MANDO_LIB=${L#A=} DEPTH=60 LEN_LO=7000 LEN_HI=8000 timeout -k 10 300 python tools/prof.py 16 2>&1 | grep -E "fast rows|cycles per read|refills|^groups" | cut -c1-200
done
timeout -k 10 400 python bench.py --workload config5 --steps 1 --warmup 1 --no-cpu-baseline > $D/c5.json 2> $D/c5.err || { tail -20 $D/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/c5.json')); print('config5', d['ms_per_step'], d['config']['phases_rank0_s'])"
