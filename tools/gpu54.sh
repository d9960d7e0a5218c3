# r01 s5: compact factor rows in the bucketed Sinkhorn (LDS-resident up to 1202 points): loss parity + timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_loss.py > gpurun_out/t54_tests.log 2>&1 || { tail -40 gpurun_out/t54_tests.log; exit 1; }
tail -1 gpurun_out/t54_tests.log
timeout -k 10 200 python -u tools/loss_probe.py > gpurun_out/t54_probe.log 2>&1 || { tail -20 gpurun_out/t54_probe.log; exit 1; }
cat gpurun_out/t54_probe.log
