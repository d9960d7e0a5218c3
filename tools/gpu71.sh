# r01 s5: eval bench refresh (config 5) after the GEMM tile retune, fp32 and fp16
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --eval --dtype fp32 --steps 5 --warmup 1 > gpurun_out/t71_eval32.log 2>&1 || { tail -20 gpurun_out/t71_eval32.log; exit 1; }
tail -1 gpurun_out/t71_eval32.log
timeout -k 10 300 python -u bench.py --eval --dtype fp16 --steps 10 --warmup 2 > gpurun_out/t71_eval16.log 2>&1 || { tail -20 gpurun_out/t71_eval16.log; exit 1; }
tail -1 gpurun_out/t71_eval16.log
