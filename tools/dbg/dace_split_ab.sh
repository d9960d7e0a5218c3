#!/bin/bash
# DACE loss A/B by kernel trace (per call span, tools/dbg/dace_split_ab.py): for each library build in LIBS (directories
# holding libebc_hip.so), interleaved over 2 rounds.  TAG names the output gpurun_out/TAG_dace_split.txt.
O=$PWD/gpurun_out; R=$PWD; mkdir -p $O
for r in 1 2; do
  for L in $LIBS; do
    n=$(basename $L); d=$O/${TAG}_ds_${n}_$r
    (cd /tmp && export TMPDIR=/tmp && EBC_LIB_PATH=$R/$L/libebc_hip.so timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run -- \
      python3 $R/tools/dbg/dace_split_ab.py run > $d.log 2>&1) || { tail -20 $d.log; exit 1; }
    db=$(find $d -name "*.db" | head -1)
    echo "== $n round $r" >> $O/${TAG}_dace_split.txt
    python3 $R/tools/dbg/dace_split_ab.py parse "$db" >> $O/${TAG}_dace_split.txt || exit 1
    rm -rf $d
  done
done
cat $O/${TAG}_dace_split.txt
