#!/bin/bash
# Decoder conv GEMM tile / split sweep at the bench shape (tools/conv_bench.py per setting) -> gpurun_out/TAG_conv_sweep.txt
TAG=${1:?tag}; O=gpurun_out; mkdir -p $O; T=$O/${TAG}_conv_sweep.txt; : > $T
for r in 1 2; do
  for cs in ${CONV_SWEEP:-"auto:" "3:1" "3:2" "3:4" "7:1" "7:2" "7:3" "13:1" "13:2" "20:1" "20:3" "21:1" "21:2"}; do
    c=${cs%%:*}; s=${cs##*:}
    envs=""; [ "$c" != auto ] && envs="EBC_CONV_CFG=$c"; [ -n "$s" ] && envs="$envs EBC_CONV_SPLITS=$s"
    out=$(timeout -k 10 120 env $envs python -u tools/conv_bench.py 2>&1 | tail -1) || { echo "FAILED $cs: $out"; exit 1; }
    echo "r$r cfg=$c splits=${s:-plan}: $out" | tee -a $T
  done
done
