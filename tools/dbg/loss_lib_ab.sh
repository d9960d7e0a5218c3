#!/bin/bash
# interleaved rounds of tools/dbg/loss_lib_ab.py over the library builds in LIBS (directories holding libebc_hip.so)
O=gpurun_out; mkdir -p $O
for r in 1 2; do
  for L in $LIBS; do
    EBC_LIB_PATH=$PWD/$L/libebc_hip.so timeout -k 10 120 python -u tools/dbg/loss_lib_ab.py >> $O/${TAG}_loss_ab.txt 2>&1 || exit 1
  done
done
grep " us " $O/${TAG}_loss_ab.txt
