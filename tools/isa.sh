#!/bin/bash
# Disassemble the gfx950 code object of a hipcc object:  tools/isa.sh build/attention.o OUT.s
set -e
o=$(readlink -f "$1"); t=$(mktemp -d)
objcopy --dump-section .hip_fatbin=$t/fb.bin "$o" $t/copy.o   # explicit output: never rewrite the input
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$t/fb.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$t/k.co
/opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn $t/k.co > "$2"
rm -rf $t
