# r01 s5: loss kernel per-crop cycles vs point count (is the Sinkhorn loop work- or latency-bound?)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/loss_prof.py 1 10 40 100 200 300 450 > gpurun_out/t52_lossprof.log 2>&1 || { tail -20 gpurun_out/t52_lossprof.log; exit 1; }
cat gpurun_out/t52_lossprof.log | tail -60
