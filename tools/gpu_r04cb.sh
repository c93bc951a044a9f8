# GPU box: config-4 chunk size A/B (MANDO_CHUNK_BYTES in GiB, GBS), interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04cb}
mkdir -p $D
G=1073741824
for rep in 1 2; do
  for gb in ${GBS:-4 2 3 6}; do
    name=c4_${gb}g_$rep
    MANDO_CHUNK_BYTES=$(python3 -c "print(int($gb * $G))") timeout -k 10 600 python3 bench.py --workload config4 --steps 3 --warmup 1 --no-cpu-baseline > $D/$name.json 2> $D/$name.err || { echo "$name failed"; tail -5 $D/$name.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/$name.json')); c=d['config']; print('$name', round(d['ms_per_step'], 1), c['steps_s'], c['steps_poa_kernel_ms'], c.get('chunks'), c['full_output_equals_oracle'])"
  done
done
