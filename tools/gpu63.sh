# r01 s5: re-sweep the GEMM tile configs at the ViT shapes with the current kernel (is pick_cfg still right?)
set -o pipefail
mkdir -p gpurun_out
for c in 0 2 4 5 8 9 12 13 3 6 10 11 1 20 21 22 24; do
  echo "== cfg $c" >> gpurun_out/t63_sweep.log
  EBC_GEMM_CFG=$c timeout -k 10 120 python tools/gemm_bench.py >> gpurun_out/t63_sweep.log 2>&1 || { tail -20 gpurun_out/t63_sweep.log; exit 1; }
done
echo done
