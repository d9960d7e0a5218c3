# r01: sliding-window eval benchmark (config 5), fp32 (reference precision) and fp16
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --eval --steps 3 --warmup 1 --dtype fp32 > gpurun_out/t38_eval32.log 2>&1 || { tail -20 gpurun_out/t38_eval32.log; exit 1; }
tail -1 gpurun_out/t38_eval32.log
timeout -k 10 300 python -u bench.py --eval --steps 5 --warmup 2 --dtype fp16 > gpurun_out/t38_eval16.log 2>&1 || { tail -20 gpurun_out/t38_eval16.log; exit 1; }
tail -1 gpurun_out/t38_eval16.log
