set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_model.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t7_tests.log 2>&1 || { tail -30 gpurun_out/t7_tests.log; exit 1; }
for c in 3 13 20 21 2; do EBC_CONV_CFG=$c timeout -k 10 60 python -u tools/conv_bench.py >> gpurun_out/t7_conv.log 2>&1 || exit 1; done
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/t7_bench.log 2>&1
