#!/bin/bash
# GEMM / conv anatomy on the box (r06): the timeline labs built with the gemm.hip lab switches (tools/lab/bin/
# {conv,gemm}_tl_{base,nomfma,noload,noepi,skel}), then two rocprofv3 --pmc passes over each base lab (stall / LDS
# counters, MFMA / VALU / L2 counters), summarised per kernel by tools/pmc.py.   TAG names the outputs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
T=$O/${TAG}_anatomy.txt; : > $T
for lab in conv gemm; do
  for v in base nomfma noload noepi skel; do
    echo "== ${lab}_tl_$v" >> $T
    timeout -k 10 120 $R/tools/lab/bin/${lab}_tl_$v 5 > $O/${TAG}_${lab}_$v.txt 2>&1 || { tail -20 $O/${TAG}_${lab}_$v.txt; exit 1; }
    grep -E "tiles|segments|k-loop|epilogue|prologue" $O/${TAG}_${lab}_$v.txt >> $T
  done
done
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  for lab in conv gemm; do
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $O/${TAG}_pmc_${lab}_$i -o run -- \
      $R/tools/lab/bin/${lab}_tl_base 2 > $O/${TAG}_pmc_${lab}_$i.log 2>&1) || { tail -20 $O/${TAG}_pmc_${lab}_$i.log; exit 1; }
    db=$(find $O/${TAG}_pmc_${lab}_$i -name "*.db" | head -1)
    echo "== pmc pass $i $lab" >> $T
    python3 $R/tools/pmc.py "$db" >> $T || exit 1
    rm -rf $O/${TAG}_pmc_${lab}_$i
  done
done
cat $T
