# Dev: end-to-end D module at config-3 size for several chunk counts (tools/e2e_timeline.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/chunks
export TMPDIR=/tmp
for c in ${CHUNK_LIST:-2 3 4 6 8}; do
  CHUNKS=$c timeout -k 10 300 python -u tools/e2e_timeline.py 20000 > gpurun_out/chunks/c$c.log 2>&1 || exit 1
  echo "chunks $c: $(grep t_total gpurun_out/chunks/c$c.log)"
done
