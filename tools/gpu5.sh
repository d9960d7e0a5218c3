set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/torch_prof.py > gpurun_out/t5_torchprof.log 2>&1
