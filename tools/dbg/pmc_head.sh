#!/bin/bash
# the similarity head (tools/kbench.py head 16) under two PMC passes, summarised per kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "FETCH_SIZE SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $O/r04ze_pmc$i -o run -- python3 $R/tools/kbench.py head 16 --reps 20 > $O/r04ze_pmc$i.log 2>&1) || { tail -20 $O/r04ze_pmc$i.log; exit 1; }
  db=$(find $O/r04ze_pmc$i -name "*.db" | head -1)
  python3 $R/tools/pmc.py "$db" --match head > $O/r04ze_pmc$i.txt || exit 1
  rm -rf $O/r04ze_pmc$i
done
cat $O/r04ze_pmc1.txt $O/r04ze_pmc2.txt $O/r04ze_pmc3.txt | sed 's/_ZN[^ ]*//' 
