# r01: 256x96 split-K tiles (cfg 32) for the N=768 GEMMs; order-free 2-split sum
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py > gpurun_out/t32_tests.log 2>&1 || { tail -40 gpurun_out/t32_tests.log; exit 1; }
tail -1 gpurun_out/t32_tests.log
for v in "" "EBC_GEMM_CFG=32" "EBC_GEMM_CFG=32 EBC_GEMM_SPLITS=3" "EBC_GEMM_CFG=21" ""; do
  echo "== $v"
  env $v timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 120 python tools/conv_bench.py 2>&1 | grep -v amdgpu.ids
