set -o pipefail
mkdir -p gpurun_out
for nw in 8 16; do echo "NW=$nw" >> gpurun_out/t14_attn.log; EBC_ATTN_NW=$nw timeout -k 10 60 python -u tools/attn_bench.py >> gpurun_out/t14_attn.log 2>&1 || exit 1; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k attention --timeout 120 --timeout-method thread > gpurun_out/t14_tests.log 2>&1; tail -2 gpurun_out/t14_tests.log
