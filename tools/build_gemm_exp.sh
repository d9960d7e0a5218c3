#!/bin/bash
# Experiment builds of libebc_hip.so for GEMM bottleneck analysis (tools/gemm_bench.py with
# EBC_LIB_PATH=clip-ebc_amd/lib/exp<m>/libebc_hip.so):  1 = no MFMA, 2 = no global->LDS loads, 4 = no epilogue (bits combine).
set -e
cd "$(dirname "$0")/../clip-ebc_amd"
for m in "$@"; do
  mkdir -p build/exp$m lib/exp$m
  for f in csrc/*.hip; do
    o=build/exp$m/$(basename "${f%.hip}").o
    extra=""; [ "$(basename $f)" = gemm.hip ] && extra="-mllvm -amdgpu-mfma-vgpr-form=1 -DEBC_GEMM_EXP=$m"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics $extra -c $f -o $o &
  done
  wait
  /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o lib/exp$m/libebc_hip.so build/exp$m/*.o
done
