#!/bin/bash
# PMC passes over tools/attn_bench.py (isolated attention kernels at the bench shape) -> gpurun_out/TAG_attn_pmc.txt
set -o pipefail
TAG=${1:?tag}; R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $O/${TAG}_apmc$i -o run -- \
    python3 $R/tools/attn_bench.py > $O/${TAG}_apmc$i.log 2>&1) || { tail -20 $O/${TAG}_apmc$i.log; exit 1; }
done
for i in 1 2; do db=$(find $O/${TAG}_apmc$i -name "*.db" | head -1); python3 $R/tools/pmc.py "$db" --match attn; done > $O/${TAG}_attn_pmc.txt
rm -rf $O/${TAG}_apmc1 $O/${TAG}_apmc2
cat $O/${TAG}_attn_pmc.txt
