# r01: persistent loop reverted, split-K sum in split order without re-reads, bn_bwd_partial / vpt_grad rewrites
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_decoder.py tests/test_gpu_model.py tests/test_gpu_kernels.py > gpurun_out/t31_tests.log 2>&1 || { tail -40 gpurun_out/t31_tests.log; exit 1; }
tail -2 gpurun_out/t31_tests.log
timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python tools/conv_bench.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/t31_bench.log 2>&1 || exit 1
tail -1 gpurun_out/t31_bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/t31_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/t31_prof.log 2>&1
