#!/bin/bash
# Same-box A/B of library builds on the bench step (interleaved runs, no probe / CPU baseline):
#   tools/ab_bench.sh TAG "bench args" lib1 lib2 ...   (lib = a directory under clip-ebc_amd/lib, "." = the default)
set -o pipefail
TAG=$1; ARGS=$2; shift 2
O=gpurun_out; mkdir -p $O; T=$O/${TAG}_ab.txt; : > $T
for r in 1 2; do
  for l in "$@"; do
    timeout -k 10 300 env EBC_LIB_PATH=clip-ebc_amd/lib/$l/libebc_hip.so python -u bench.py $ARGS --no-cpu-baseline --no-probe \
      > $O/${TAG}_ab_last.log 2>&1 || { echo "FAILED $l"; tail -20 $O/${TAG}_ab_last.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/${TAG}_ab_last.log').read().strip().splitlines()[-1]); print('$l', d['value'], d['ms_per_step'], d.get('median_ms_per_step'))" | tee -a $T
  done
done
