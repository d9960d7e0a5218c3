# r01 s5: refresh the roofline traffic of the bench's dominant kernel (c_fc + GELU, 3664x3072x768): separate PMC passes
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/t74_pmc_fetch -o run -- python3 $R/tools/gemm_one.py 3664 3072 768 1 > $R/gpurun_out/t74_pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/t74_pmc_write -o run -- python3 $R/tools/gemm_one.py 3664 3072 768 1 > $R/gpurun_out/t74_pmc_write.log 2>&1 || exit 1
echo ok
