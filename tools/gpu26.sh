# r01: direct-from-register GEMM epilogue: GEMM + model parity, GEMM bench, train bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_model.py > gpurun_out/t26_tests.log 2>&1 || { tail -40 gpurun_out/t26_tests.log; exit 1; }
tail -2 gpurun_out/t26_tests.log
timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/t26_gemm.log 2>&1 || exit 1
cat gpurun_out/t26_gemm.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/t26_bench.log 2>&1 || exit 1
tail -1 gpurun_out/t26_bench.log | cut -c1-200
