#!/bin/bash
# Isolated A/B of GEMM variants on the box (tools/kbench.py, interleaved rounds), output -> gpurun_out/$1.txt
set -o pipefail
O=gpurun_out; mkdir -p $O; T=$O/$1.txt; : > $T
N768="gemm:3664,768,3072,2 gemm:3664,768,3072,0 gemm:3664,768,2304,0 gemm:3664,768,768,2"
WIDE="gemm:3664,3072,768,3 gemm:3664,3072,768,1 gemm:3664,2304,768,0"
run() { echo "== $*" >> $T; timeout -k 10 120 env "$@" >> $T 2>&1 || { echo "FAILED $*" >> $T; exit 1; }; }
run X=0 python tools/kbench.py multi $N768 $WIDE --reps 50 --rounds 2
run EBC_GEMM_CFG=14 EBC_GEMM_SPLITS=2 python tools/kbench.py multi $N768 --reps 50 --rounds 2
run EBC_GEMM_CFG=14 EBC_GEMM_SPLITS=1 python tools/kbench.py multi $N768 --reps 50 --rounds 1
run EBC_GEMM_CFG=3 EBC_GEMM_SPLITS=4 python tools/kbench.py multi $N768 --reps 50 --rounds 2
run EBC_GEMM_CFG=3 EBC_GEMM_SPLITS=2 python tools/kbench.py multi $N768 --reps 50 --rounds 1
run EBC_GEMM_CFG=6 EBC_GEMM_SPLITS=2 python tools/kbench.py multi $N768 --reps 50 --rounds 1
for v in e1 e2 v_a1 v_a2 v_a3 v_a16; do
  run EBC_LIB_PATH=clip-ebc_amd/lib/$v/libebc_hip.so python tools/kbench.py multi $N768 $WIDE --reps 50 --rounds 2
done
run X=1 python tools/kbench.py multi $N768 $WIDE --reps 50 --rounds 1
cat $T
