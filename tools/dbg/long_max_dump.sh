#!/bin/bash
# tools/dbg/long_max_dump.py over the lab builds of the failing long-attention ordering (r06): lmbad (no hook), lmbadd
# (per-chunk dump: the failure disappears), lmbade (end-of-kernel dump), lmgoodd (the shipped ordering, per-chunk dump)
set -o pipefail
O=gpurun_out; mkdir -p $O; T=$O/${TAG:-r06s}_long_max.txt
for v in ${VARS:-lmbad lmbadd lmgoodd}; do
  echo "== $v" >> $T
  EBC_LIB_PATH=clip-ebc_amd/lib/$v/libebc_hip.so timeout -k 10 120 python -u tools/dbg/long_max_dump.py >> $T 2>&1 || exit 1
done
cat $T
