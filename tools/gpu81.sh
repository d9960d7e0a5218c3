# r01 s5: projection GEMM tile sweep at the eval batch (M = 140 x 784 = 109760 pixel rows)
set -o pipefail
mkdir -p gpurun_out
for c in 0 1 2 6 7 10 21 22; do
  echo "== cfg $c" >> gpurun_out/t81_sweep.log
  GB_SET=proj GB_M=109760 EBC_GEMM_CFG=$c timeout -k 10 120 python tools/gemm_bench.py >> gpurun_out/t81_sweep.log 2>&1 || { tail -20 gpurun_out/t81_sweep.log; exit 1; }
done
echo done
