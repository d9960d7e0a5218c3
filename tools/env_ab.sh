#!/bin/bash
# Same-box A/B of an environment switch on the bench step (interleaved runs, no probe / CPU baseline):
#   tools/env_ab.sh TAG "bench args" "ENV=a" "ENV=b" ...
set -o pipefail
TAG=$1; ARGS=$2; shift 2
O=gpurun_out; mkdir -p $O; T=$O/${TAG}_envab.txt; : > $T
for r in 1 2; do
  for e in "$@"; do
    timeout -k 10 300 env $e python -u bench.py $ARGS --no-cpu-baseline --no-probe > $O/${TAG}_envab_last.log 2>&1 \
      || { echo "FAILED $e"; tail -20 $O/${TAG}_envab_last.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/${TAG}_envab_last.log').read().strip().splitlines()[-1]); print('$e', d['value'], d['ms_per_step'], d.get('median_ms_per_step'))" | tee -a $T
  done
done
