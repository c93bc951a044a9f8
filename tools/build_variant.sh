#!/bin/bash
# Dev helper: build libmando.so with extra compile flags into build/<name>/libmando.so
# usage: bash tools/build_variant.sh NAME "-DFLAG ..."   (then MANDO_LIB=build/NAME/libmando.so)
set -e
name=$1; flags=$2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/build/$name
mkdir -p $out/obj
cd $root/mandalorion_amd/csrc
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -munsafe-fp-atomics $flags"
objs=""
for f in capi.hip poa_kernel.hip orient_kernel.hip; do $H -c $f -o $out/obj/$f.o & objs="$objs $out/obj/$f.o"; done
for f in rng.cpp cluster.cpp psl.cpp sam.cpp module_f.cpp; do $H -x c++ -c $f -o $out/obj/$f.o & objs="$objs $out/obj/$f.o"; done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libmando.so $objs -lpthread -lz
echo "built $out/libmando.so"
