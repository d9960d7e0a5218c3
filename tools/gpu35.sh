# r01: Sinkhorn phase B two points per lane group, adaptive K^T u candidate rounds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_loss.py > gpurun_out/t35_tests.log 2>&1 || { tail -40 gpurun_out/t35_tests.log; exit 1; }
tail -1 gpurun_out/t35_tests.log
timeout -k 10 200 python tools/loss_prof.py 4 20 100 250 400 > gpurun_out/t35_loss_prof.log 2>&1 || { tail -20 gpurun_out/t35_loss_prof.log; exit 1; }
grep -E "^---|crop 0" gpurun_out/t35_loss_prof.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/t35_bench.log 2>&1 || exit 1
tail -1 gpurun_out/t35_bench.log | cut -c1-200
