# r01 s5: eval bench with 256-wide tiles for the many-tile eval shapes, fp32 and fp16
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_eval.py tests/test_gpu_model.py > gpurun_out/t73_tests.log 2>&1 || { tail -30 gpurun_out/t73_tests.log; exit 1; }
tail -1 gpurun_out/t73_tests.log
timeout -k 10 300 python -u bench.py --eval --dtype fp32 --steps 5 --warmup 1 > gpurun_out/t73_eval32.log 2>&1 || { tail -20 gpurun_out/t73_eval32.log; exit 1; }
tail -1 gpurun_out/t73_eval32.log
timeout -k 10 300 python -u bench.py --eval --dtype fp16 --steps 10 --warmup 2 > gpurun_out/t73_eval16.log 2>&1 || { tail -20 gpurun_out/t73_eval16.log; exit 1; }
tail -1 gpurun_out/t73_eval16.log
