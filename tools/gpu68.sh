# r01 s5: decoder conv GEMM sweep (tile config x split-K for the weight gradient)
set -o pipefail
mkdir -p gpurun_out
for c in 3 13 20 21; do
  for s in 0 1 2 3 4 6; do
    echo "== cfg $c splits $s" >> gpurun_out/t68_sweep.log
    EBC_CONV_CFG=$c EBC_CONV_SPLITS=$s timeout -k 10 120 python tools/conv_bench.py >> gpurun_out/t68_sweep.log 2>&1 || { tail -20 gpurun_out/t68_sweep.log; exit 1; }
  done
done
echo done
