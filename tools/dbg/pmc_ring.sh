#!/bin/bash
# ring_lab under two PMC passes (LDS / SQ counters), summarised per kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
i=0
for ctrs in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $O/r04z_pmc$i -o run -- $R/tools/lab/bin/ring_lab 1 5 > $O/r04z_pmc$i.log 2>&1) || { tail -20 $O/r04z_pmc$i.log; exit 1; }
  db=$(find $O/r04z_pmc$i -name "*.db" | head -1)
  python3 $R/tools/pmc.py "$db" --match gemm_nt > $O/r04z_pmc$i.txt || exit 1
  rm -rf $O/r04z_pmc$i
done
cat $O/r04z_pmc1.txt $O/r04z_pmc2.txt
