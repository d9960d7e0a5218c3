set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --kernel-trace -d $R/gpurun_out/t17_pmc1 -o run -- python3 $R/tools/gemm_one.py 3664 3072 768 1 > $R/gpurun_out/t17_pmc1.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $R/gpurun_out/t17_pmc2 -o run -- python3 $R/tools/gemm_one.py 3664 3072 768 1 > $R/gpurun_out/t17_pmc2.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --kernel-trace -d $R/gpurun_out/t17_pmc3 -o run -- python3 $R/tools/conv_bench.py > $R/gpurun_out/t17_pmc3.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $R/gpurun_out/t17_pmc4 -o run -- python3 $R/tools/conv_bench.py > $R/gpurun_out/t17_pmc4.log 2>&1
