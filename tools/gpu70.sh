# r01 s5: new tile configs (14: 128x96 S4, 15: 128x96/8w S3, 18: 192x192/8w S3) vs the defaults at the ViT shapes
set -o pipefail
mkdir -p gpurun_out
for c in 0 13 14 15 4 18; do
  echo "== cfg $c" >> gpurun_out/t70_sweep.log
  EBC_GEMM_CFG=$c timeout -k 10 120 python tools/gemm_bench.py >> gpurun_out/t70_sweep.log 2>&1 || { tail -20 gpurun_out/t70_sweep.log; exit 1; }
done
echo done
