# r01 s5: attention waves per workgroup (8 vs 16) at 16 / 32 crops and the 140-tile eval batch
set -o pipefail
mkdir -p gpurun_out
for b in 16 32 140; do
  for nw in 16 8; do
    echo "== B $b NW $nw" >> gpurun_out/t82.log
    AB=$b EBC_ATTN_NW=$nw timeout -k 10 120 python tools/attn_bench.py >> gpurun_out/t82.log 2>&1 || { tail -20 gpurun_out/t82.log; exit 1; }
  done
done
echo done
