#!/bin/bash
# Dev helper: build libmando.so with extra compile flags into build/<name>/libmando.so
# usage: bash tools/build_variant.sh NAME "-DFLAG ..."   (then MANDO_LIB=build/NAME/libmando.so)
set -e
name=$1; flags=$2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/${VARIANT_DIR:-build}/$name
mkdir -p $out
make -s -j8 -C $root/mandalorion_amd/csrc OUT=$out "HIPFLAGS=--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -munsafe-fp-atomics $flags" $out/libmando.so
echo "built $out/libmando.so"
