set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for w in config2 config5; do
for v in "X=0" "MANDO_CHUNKS=1"; do
  env $v timeout -k 10 400 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > /tmp/b.json 2> /tmp/b.err || { tail -5 /tmp/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('/tmp/b.json')); print('$w $v', round(d['ms_per_step']), d['config']['phases_rank0_s'])"
done; done
