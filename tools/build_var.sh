#!/bin/bash
# Variant builds of libebc_hip.so with extra defines on ONE source file, for same-box A/B (tools/ab_bench.sh,
# EBC_LIB_PATH=clip-ebc_amd/lib/<name>/libebc_hip.so); the other objects come from the regular build (run make first):
#   tools/build_var.sh <source stem[,stem2...]> name1 "-DX=1" [name2 "-DX=2" ...]      e.g. tools/build_var.sh prefetch pf0 "-DEBC_PREFETCH_WGS=0"
set -e
cd "$(dirname "$0")/../clip-ebc_amd"
IFS=, read -ra srcs <<< "$1"; shift
args=("$@")
for ((i = 0; i < ${#args[@]}; i += 2)); do
  n=${args[i]}; d=${args[i+1]}
  mkdir -p build/$n lib/$n
  for src in "${srcs[@]}"; do
    FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics"
    [ "$src" = gemm ] && FLAGS="$FLAGS -mllvm -amdgpu-mfma-vgpr-form=1"
    /opt/rocm/bin/hipcc $FLAGS $d -c csrc/$src.hip -o build/$n/$src.o &
  done
done
wait
for ((i = 0; i < ${#args[@]}; i += 2)); do
  n=${args[i]}
  objs=""
  for o in build/*.o; do
    b=$(basename $o .o); [ -f build/$n/$b.o ] && objs="$objs build/$n/$b.o" || objs="$objs $o"
  done
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o lib/$n/libebc_hip.so $objs
done
