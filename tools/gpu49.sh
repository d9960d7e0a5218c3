# r01: torch-profiler attribution of the remaining copies / fills (call stacks)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/torch_prof.py --steps 3 > gpurun_out/t49_torchprof.log 2>&1 || { tail -20 gpurun_out/t49_torchprof.log; exit 1; }
grep -A200 "== copy/fill ops by call stack" gpurun_out/t49_torchprof.log | head -120
