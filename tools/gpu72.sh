# r01 s5: tile sweep at the eval batch (M = 140 tiles x 229 tokens = 32060 rows)
set -o pipefail
mkdir -p gpurun_out
for c in 0 2 3 4 5 13 6 7 10 1 9 20 21 22; do
  echo "== cfg $c" >> gpurun_out/t72_sweep.log
  GB_M=32060 EBC_GEMM_CFG=$c timeout -k 10 120 python tools/gemm_bench.py >> gpurun_out/t72_sweep.log 2>&1 || { tail -20 gpurun_out/t72_sweep.log; exit 1; }
done
echo done
