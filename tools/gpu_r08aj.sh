# Config 4 end to end, interleaved: the previous POA kernel (abv/base) against the in-tree one, bench.py
# --steps 5 each, twice (no CPU baseline), one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r08aj}
mkdir -p $D
for pass in 1 2; do
  for v in base head; do
    lib=abv/base/libmando.so; [ $v = head ] && lib=mandalorion_amd/lib/libmando.so
    MANDO_LIB=$lib timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $D/$v.$pass.json 2> $D/$v.$pass.err || { echo "$v.$pass failed"; tail -5 $D/$v.$pass.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/$v.$pass.json')); c=d['config']; print('$v.$pass', round(d['ms_per_step']), c['steps_s'], c['steps_poa_kernel_ms'], c['full_output_equals_oracle'])"
  done
done
