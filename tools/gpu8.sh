set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_decoder.py tests/test_gpu_model.py -q --timeout 120 --timeout-method thread > gpurun_out/t8_tests.log 2>&1 || { tail -40 gpurun_out/t8_tests.log; exit 1; }
tail -2 gpurun_out/t8_tests.log
timeout -k 10 200 python -u tools/loss_probe.py > gpurun_out/t8_loss_probe.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/loss_prof.py > gpurun_out/t8_loss_prof.log 2>&1 || exit 1
for c in 3 13 20 21; do EBC_CONV_CFG=$c timeout -k 10 60 python -u tools/conv_bench.py >> gpurun_out/t8_conv.log 2>&1 || exit 1; done
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/t8_bench.log 2>&1
tail -1 gpurun_out/t8_bench.log | cut -c1-200
