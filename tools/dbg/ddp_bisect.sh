#!/bin/bash
# The world-2 DDP + SyncBN GPU test on several library builds (default: r03 final, r04 compact-K, the tree's; LIBS
# overrides the list).  Each entry is a directory holding a libebc_hip.so built from a git worktree (not committed).
O=gpurun_out; mkdir -p $O
for L in ${LIBS:-tools/dbg/lib_r03 tools/dbg/lib_r04b clip-ebc_amd/lib}; do
  echo "== $L" >> $O/${TAG:-r04i}_ddp.txt
  EBC_LIB_PATH=$PWD/$L/libebc_hip.so timeout -k 10 200 python -u -m pytest -x -q -s --timeout 180 --timeout-method thread \
    -m gpu tests/test_gpu_ddp.py >> $O/${TAG:-r04i}_ddp.txt 2>&1
  rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
grep -E "^==|worst|passed|failed" $O/${TAG:-r04i}_ddp.txt
