#!/bin/bash
# Same-box A/B of bench.py argument sets (interleaved, two rounds, no probe / CPU baseline):
#   tools/ab_args.sh TAG "args A" "args B" ...
set -o pipefail
TAG=$1; shift
O=gpurun_out; mkdir -p $O; T=$O/${TAG}_ab.txt; : > $T
for r in 1 2; do
  for a in "$@"; do
    timeout -k 10 300 python -u bench.py $a --no-cpu-baseline --no-probe > $O/${TAG}_ab_last.log 2>&1 \
      || { echo "FAILED $a"; tail -20 $O/${TAG}_ab_last.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/${TAG}_ab_last.log').read().strip().splitlines()[-1]); print('[$a]', d['value'], d['ms_per_step'], d.get('median_ms_per_step'))" | tee -a $T
  done
done
