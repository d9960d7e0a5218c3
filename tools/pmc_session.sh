#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, each under its own hard time limit) over single kernel
# classes run by tools/kbench.py; summaries -> gpurun_out/pmc_<tag>_*.json (tools/pmc.py).
# usage (on the box, repo root): tools/pmc_session.sh TAG "gemm 3664 768 3072 2" ["attn 16" ...]
set -o pipefail
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
PASSES=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_F16"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
)
cd /tmp && export TMPDIR=/tmp
k=0
for spec in "$@"; do
  k=$((k+1))
  p=0
  for ctrs in "${PASSES[@]}"; do
    p=$((p+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctrs -d $O/k${k}_p${p} -o run -- python3 $R/tools/kbench.py $spec --reps 10 \
      > $O/k${k}_p${p}.log 2>&1 || { echo "pass $p of [$spec] failed"; tail -5 $O/k${k}_p${p}.log; exit 1; }
  done
  python3 $R/tools/pmc.py --merge $O/k${k}_p*/ --label "$spec" --json $O/k${k}.json > $O/k${k}.txt || exit 1
  cat $O/k${k}.txt
  rm -rf $O/k${k}_p*/                 # the databases are large; the merged JSON keeps what is read
done
echo "pmc_session $TAG done"
