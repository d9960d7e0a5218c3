set -o pipefail
mkdir -p gpurun_out
EBC_GEMM_CFG=27 EBC_CONV_CFG=27 timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_decoder.py -q --timeout 120 --timeout-method thread > gpurun_out/t18_tests.log 2>&1; tail -3 gpurun_out/t18_tests.log
for c in 3 27; do EBC_CONV_CFG=$c timeout -k 10 60 python -u tools/conv_bench.py >> gpurun_out/t18_conv.log 2>&1 || exit 1; done
for c in 3 4 27; do echo "== cfg $c" >> gpurun_out/t18_gemm.log; EBC_GEMM_CFG=$c timeout -k 10 60 python -u tools/gemm_bench.py >> gpurun_out/t18_gemm.log 2>&1 || exit 1; done
