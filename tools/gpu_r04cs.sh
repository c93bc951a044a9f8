# GPU box: chunk size 4 vs 6 GiB on rank 0's share of the 2- and 4-rank config-4 plans, interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04cs}
mkdir -p $D
G=1073741824
for rep in 1 2; do
  for sh in 2 4; do
    for gb in 4 6; do
      name=s${sh}_${gb}g_$rep
      MANDO_CHUNK_BYTES=$((gb * G)) timeout -k 10 600 python3 bench.py --workload config4 --share $sh --steps 3 --warmup 1 --no-cpu-baseline > $D/$name.json 2> $D/$name.err || { echo "$name failed"; tail -5 $D/$name.err; exit 1; }
      python3 -c "import json; d=json.load(open('$D/$name.json')); c=d['config']; print('$name', round(d['ms_per_step'], 1), c['steps_s'], c['steps_poa_kernel_ms'], c.get('chunks'))"
    done
  done
done
