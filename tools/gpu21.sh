set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t22_tests.log 2>&1 || { tail -30 gpurun_out/t22_tests.log; exit 1; }
tail -1 gpurun_out/t22_tests.log
timeout -k 10 60 python -u tools/gemm_bench.py > gpurun_out/t22_gemm.log 2>&1 || exit 1
timeout -k 10 60 python -u tools/conv_bench.py > gpurun_out/t22_conv.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/t22_bench.log 2>&1 || exit 1
tail -1 gpurun_out/t22_bench.log | cut -c1-150
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/t22_bench2.log 2>&1 || exit 1
tail -1 gpurun_out/t22_bench2.log | cut -c1-150
