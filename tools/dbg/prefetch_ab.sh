#!/bin/bash
# same-box A/B of bench.py with and without the next batch's patch-embedding prefetch (interleaved, 2 rounds each)
O=gpurun_out; : > $O/${TAG}_prefetch_ab.txt
for r in 1 2; do
  for f in "--prefetch" "" "--prefetch --hiprio" "--hiprio"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-probe $f > $O/${TAG}_ab.log 2>&1 || { tail -20 $O/${TAG}_ab.log; exit 1; }
    echo "flags=${f:-none} $(tail -1 $O/${TAG}_ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["median_ms_per_step"])')" >> $O/${TAG}_prefetch_ab.txt
  done
done
cat $O/${TAG}_prefetch_ab.txt
