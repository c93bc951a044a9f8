# GPU box: POA kernel variant A/B (tools/ab_prof.sh: tools/prof.py, 20,000 config-3-shaped groups,
# interleaved twice) after the variant's POA GPU tests pass byte-exact.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r04x}
mkdir -p $D
V=${V:-rsaddr}
MANDO_LIB=variants/$V/libmando.so timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_$V.log 2>&1 || { echo "variant tests failed"; tail -30 $D/pytest_$V.log; exit 1; }
tail -1 $D/pytest_$V.log
bash tools/ab_prof.sh ${TAG:-r04x}/ab base=mandalorion_amd/lib/libmando.so $V=variants/$V/libmando.so
