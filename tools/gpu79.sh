# r01 s5: 2-stage 128x96 tiles above one wave (config-4 shape): GEMM/model tests, 32- and 16-crop bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_model.py tests/test_gpu_eval.py > gpurun_out/t79_tests.log 2>&1 || { tail -30 gpurun_out/t79_tests.log; exit 1; }
tail -1 gpurun_out/t79_tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --crops-per-gpu 32 --no-cpu-baseline > gpurun_out/t79_bench32_$r.log 2>&1 || { tail -20 gpurun_out/t79_bench32_$r.log; exit 1; }
tail -1 gpurun_out/t79_bench32_$r.log | cut -c1-200
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/t79_bench16.log 2>&1 || { tail -20 gpurun_out/t79_bench16.log; exit 1; }
tail -1 gpurun_out/t79_bench16.log | cut -c1-200
