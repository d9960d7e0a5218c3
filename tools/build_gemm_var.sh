#!/bin/bash
# Variant builds of libebc_hip.so with extra defines on gemm.hip only, for isolated A/B timing
# (tools/kbench.py with EBC_LIB_PATH=clip-ebc_amd/lib/<name>/libebc_hip.so):
#   tools/build_gemm_var.sh name1 "-DEBC_GLDS_AUX=1" name2 "-DEBC_GLDS_AUX=2" ...
# The other objects come from the regular build (run `make` first).
set -e
cd "$(dirname "$0")/../clip-ebc_amd"
args=("$@")
for ((i = 0; i < ${#args[@]}; i += 2)); do
  n=${args[i]}; d=${args[i+1]}
  mkdir -p build/$n lib/$n
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form=1 \
    $d -c csrc/gemm.hip -o build/$n/gemm.o &
done
wait
for ((i = 0; i < ${#args[@]}; i += 2)); do
  n=${args[i]}
  objs=$(ls build/*.o | grep -v "/gemm.o")
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o lib/$n/libebc_hip.so $objs build/$n/gemm.o
done
