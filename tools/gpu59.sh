# r01 s5: GPU augmentation (f2) parity vs the CPU oracle
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_augment.py > gpurun_out/t59_tests.log 2>&1 || { tail -60 gpurun_out/t59_tests.log; exit 1; }
tail -3 gpurun_out/t59_tests.log
