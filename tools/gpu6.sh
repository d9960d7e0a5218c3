set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/loss_probe.py > gpurun_out/t6_loss_probe.log 2>&1 && \
timeout -k 10 200 python -u tools/loss_prof.py > gpurun_out/t6_loss_prof.log 2>&1
