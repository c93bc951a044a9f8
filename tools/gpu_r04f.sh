# GPU box: config 4 at HEAD (4 GiB chunks, per-kind workspace grants, backpressure), then the per-rank
# loads of 2/4/8-rank LPT plans of config 4 and config 3, each run alone on this GPU (bench.py --share).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04f}
mkdir -p $D
MANDO_WS_LOG=1 timeout -k 10 900 python3 bench.py --no-cpu-baseline --workload config4 --steps 1 --warmup 1 > $D/bench_config4.json 2> $D/bench_config4.err || { echo "config4 failed"; tail -5 $D/bench_config4.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_config4.json')); print('config4', d['value'], round(d['ms_per_step'], 1), d['config']['phases_rank0_s'])"
for w in config4 config3; do
  for n in 2 4 8; do
    st=2; [ $w = config3 ] && st=4
    timeout -k 10 600 python3 bench.py --workload $w --share $n --steps $st --warmup 1 > $D/share_${w}_$n.json 2> $D/share_${w}_$n.err || { echo "share $w $n failed"; tail -5 $D/share_${w}_$n.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/share_${w}_$n.json')); c=d['config']; print('share $w 1/$n', c['records'], round(d['ms_per_step'], 1), c['steps_s'], c['phases_rank0_s'])"
  done
done
