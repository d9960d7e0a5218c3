#!/bin/bash
# Register / spill report of the gfx950 kernels in a hipcc object:  tools/regs.sh build/gemm.o [kernel-regex]
set -e
o=$(readlink -f "$1"); t=$(mktemp -d)
objcopy --dump-section .hip_fatbin=$t/fb.bin "$o" $t/copy.o   # explicit output: never rewrite the input
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$t/fb.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$t/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $t/k.co \
  | grep -E "^\s+\.(name|vgpr_count|sgpr_count|vgpr_spill_count|private_segment_fixed_size):" \
  | awk '/\.name:/ {n=$2} !/\.name:/ {a[n]=a[n]" "$1$2} END {for (k in a) print k, a[k]}' \
  | grep -E "${2:-.}" | sed 's/\.private_segment_fixed_size:/scratch=/; s/\.sgpr_count:/sgpr=/; s/\.vgpr_count:/vgpr=/; s/\.vgpr_spill_count:/spill=/' | sort
rm -rf $t
