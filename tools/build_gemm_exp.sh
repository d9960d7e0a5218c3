#!/bin/bash
# Experiment builds of libebc_hip.so for GEMM bottleneck analysis (tools/kbench.py with
# EBC_LIB_PATH=clip-ebc_amd/lib/exp<m>/libebc_hip.so):  1 = no MFMA, 2 = no global->LDS loads, 4 = no epilogue
# (bits combine).  Only gemm.hip is rebuilt; the other objects come from the regular build (run `make` first).
set -e
cd "$(dirname "$0")/../clip-ebc_amd"
for m in "$@"; do
  mkdir -p build/exp$m lib/exp$m
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form=1 \
    -DEBC_GEMM_EXP=$m -c csrc/gemm.hip -o build/exp$m/gemm.o &
done
wait
for m in "$@"; do
  objs=$(ls build/*.o | grep -v "/gemm.o")
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o lib/exp$m/libebc_hip.so $objs build/exp$m/gemm.o
done
