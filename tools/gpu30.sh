# r01: persistent GEMM tiles (cfg 30/31, tiles per WG 1/2) and wgrad split variants
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/t30_gemm.log
for v in "" "EBC_GEMM_CFG=30" "EBC_GEMM_CFG=30 EBC_GEMM_TPW=1" "EBC_GEMM_CFG=31" "EBC_GEMM_CFG=31 EBC_GEMM_TPW=1" ""; do
  echo "== $v" >> $O
  env $v timeout -k 10 120 python tools/gemm_bench.py >> $O 2>&1 || exit 1
done
O=gpurun_out/t30_conv.log
for v in "" "EBC_CONV_SPLITS=1" "EBC_CONV_CFG=30" "EBC_CONV_CFG=30 EBC_CONV_SPLITS=2" ""; do
  echo "== $v" >> $O
  env $v timeout -k 10 120 python tools/conv_bench.py >> $O 2>&1 || exit 1
done
cat gpurun_out/t30_gemm.log | grep -v amdgpu.ids; cat gpurun_out/t30_conv.log | grep -v amdgpu.ids
