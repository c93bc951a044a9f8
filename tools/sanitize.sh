#!/bin/bash
# AddressSanitizer / ThreadSanitizer run of the CPU test suite over the host C++: libmando's host code
# (the threaded writer, PSL / SAM parsers, module F / Q, clustering host side, RNG) and the oracle
# restatements, built with clang's sanitizers into a scratch copy of the tree (the in-tree libraries are
# left alone), then `pytest -m "not gpu"` with the sanitizer runtime preloaded into Python.  GPU code is
# never sanitized (this pool refuses GPU ASan; the CPU suite makes no compute call on a GPU anyway).
# usage: bash tools/sanitize.sh address|thread [pytest args]      (this container: ~5-15 min)
set -eo pipefail
MODE=${1:-address}
shift || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/mando_san_${MODE}_XXXX)
trap 'rm -rf "$W"' EXIT
tar -C "$ROOT" --exclude=./.git --exclude=./gpurun_out --exclude=./build --exclude=./variants --exclude=./scratch \
    --exclude='*.so' --exclude='*.o' -cf - . | tar -C "$W" -xf -
LLVM=/opt/rocm/lib/llvm/bin
make -s -j8 -C "$W/mandalorion_amd/csrc" SAN=$MODE
make -s -C "$W/oracle" CC=$LLVM/clang CXX=$LLVM/clang++ SAN=$MODE
case $MODE in address) RTN=asan ;; thread) RTN=tsan ;; *) echo "mode: address or thread"; exit 1 ;; esac
RT=$($LLVM/clang -print-file-name=libclang_rt.$RTN-x86_64.so)
[ -f "$RT" ] || { echo "no sanitizer runtime $RT"; exit 1; }
cd "$W"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:symbolize=1
export TSAN_OPTIONS=halt_on_error=1:report_signal_unsafe=0:second_deadlock_stack=1:suppressions=$ROOT/tools/tsan.supp
LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}" python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider "$@"
