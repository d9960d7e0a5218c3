# r01 s5: torch-profiler attribution of copies / fills
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/torch_prof.py --steps 3 > gpurun_out/t51_torchprof.log 2>&1 || { tail -20 gpurun_out/t51_torchprof.log; exit 1; }
grep -A200 "== copy/fill ops by call stack" gpurun_out/t51_torchprof.log > gpurun_out/t51_copies.txt
