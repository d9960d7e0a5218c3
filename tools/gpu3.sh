# GEMM tile-config sweep at the ViT shapes (EBC_GEMM_CFG forces a tile config)
set -o pipefail
mkdir -p gpurun_out
for c in 2 1 3 4 6 7 10 11 13 20 21 22 24; do
  echo "== cfg $c" >> gpurun_out/t3_sweep.log
  EBC_GEMM_CFG=$c timeout -k 10 60 python -u tools/gemm_bench.py >> gpurun_out/t3_sweep.log 2>&1 || exit 1
done
