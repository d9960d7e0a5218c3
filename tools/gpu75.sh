# r01 s5: grouped tile order for the wide-N GEMMs: isolated A/B (EBC_GEMM_GROUP_M=-1 row-major vs default), PMC fetch, tests
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for r in 1 2; do
  for v in -1 0 3 6; do
    echo "== group $v run $r" >> gpurun_out/t75_ab.log
    EBC_GEMM_GROUP_M=$v timeout -k 10 120 python tools/gemm_bench.py >> gpurun_out/t75_ab.log 2>&1 || { tail -20 gpurun_out/t75_ab.log; exit 1; }
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_model.py > gpurun_out/t75_tests.log 2>&1 || { tail -30 gpurun_out/t75_tests.log; exit 1; }
tail -1 gpurun_out/t75_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/t75_pmc_fetch -o run -- python3 $R/tools/gemm_one.py 3664 3072 768 1 > $R/gpurun_out/t75_pmc_fetch.log 2>&1 || exit 1
echo ok
