#!/bin/bash
# Loss-kernel A/B by kernel trace: for each library build in LIBS (directories holding libebc_hip.so), interleaved over
# 2 rounds, rocprofv3 --kernel-trace of tools/loss_ab.py run, parsed per point-count configuration (median launch).
O=$PWD/gpurun_out; R=$PWD; mkdir -p $O
for r in 1 2; do
  for L in $LIBS; do
    n=$(basename $L); d=$O/${TAG}_kt_${n}_$r
    (cd /tmp && export TMPDIR=/tmp && EBC_LIB_PATH=$R/$L/libebc_hip.so timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run -- \
      python3 $R/tools/loss_ab.py run > $d.log 2>&1) || { tail -20 $d.log; exit 1; }
    db=$(find $d -name "*.db" | head -1)
    echo "== $n round $r" >> $O/${TAG}_loss_kt.txt
    python3 $R/tools/loss_ab.py parse "$db" >> $O/${TAG}_loss_kt.txt || exit 1
    rm -rf $d
  done
done
cat $O/${TAG}_loss_kt.txt
