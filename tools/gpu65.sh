# r01 s5: tile sweep for the 1x1 projection GEMMs (M = 16*784, N = 512 / K = 768 f32 out, N = 768 / K = 512)
set -o pipefail
mkdir -p gpurun_out
for c in 0 1 2 5 6 8 9 10 11 12 13 21 22 24; do
  echo "== cfg $c" >> gpurun_out/t65_sweep.log
  GB_SET=proj EBC_GEMM_CFG=$c timeout -k 10 120 python tools/gemm_bench.py >> gpurun_out/t65_sweep.log 2>&1 || { tail -20 gpurun_out/t65_sweep.log; exit 1; }
done
echo done
