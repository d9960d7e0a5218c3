# r01 call 2: GEMM micro-bench vs hipBLASLt, default bench (with CPU baseline), PMC traffic passes
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/gemm_bench.py > gpurun_out/t2_gemm.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/t2_bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/t2_pmc_fetch -o run -- python3 $R/tools/gemm_one.py 3664 3072 768 1 > $R/gpurun_out/t2_pmc_fetch.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/t2_pmc_write -o run -- python3 $R/tools/gemm_one.py 3664 3072 768 1 > $R/gpurun_out/t2_pmc_write.log 2>&1
