set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_loss.py -q --timeout 120 --timeout-method thread > gpurun_out/t13_tests.log 2>&1 || { tail -40 gpurun_out/t13_tests.log; exit 1; }
tail -1 gpurun_out/t13_tests.log
timeout -k 10 200 python -u tools/loss_probe.py > gpurun_out/t13_loss_probe.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/loss_prof.py > gpurun_out/t13_loss_prof.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/torch_prof.py > gpurun_out/t13_torchprof.log 2>&1
