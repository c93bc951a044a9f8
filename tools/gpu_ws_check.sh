set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; D=gpurun_out/ws1; mkdir -p $D
MANDO_WS_LOG=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $D/c3.json 2> $D/c3.err || { tail -5 $D/c3.err; exit 1; }
grep "slot workspace" $D/c3.err | sort | uniq -c | cut -c1-250
python3 -c "import json; d=json.load(open('$D/c3.json')); c=d['config']; print('c3', d['value'], c['steps_s'], c['steps_poa_kernel_ms'], c['phases_rank0_s'])"
