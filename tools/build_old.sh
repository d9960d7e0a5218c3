#!/bin/bash
# Variant build with ONE source file taken from a git revision (same-box A/B of a change against its parent):
#   tools/build_old.sh <source stem> <rev> <name>   -> clip-ebc_amd/lib/<name>/libebc_hip.so (other objects: the regular build)
set -e
cd "$(dirname "$0")/../clip-ebc_amd"
src=$1; rev=$2; n=$3
mkdir -p build/$n lib/$n
git show $rev:clip-ebc_amd/csrc/$src.hip > csrc/_old_$src.hip
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics"
[ "$src" = gemm ] && FLAGS="$FLAGS -mllvm -amdgpu-mfma-vgpr-form=1"
[ "$src" = attention ] && FLAGS="$FLAGS -fno-slp-vectorize"   # as the Makefile
/opt/rocm/bin/hipcc $FLAGS -c csrc/_old_$src.hip -o build/$n/$src.o; rm -f csrc/_old_$src.hip
objs=""
for o in build/*.o; do b=$(basename $o .o); [ -f build/$n/$b.o ] && objs="$objs build/$n/$b.o" || objs="$objs $o"; done
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o lib/$n/libebc_hip.so $objs
