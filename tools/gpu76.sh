# r01 s5: head kernels with the pixel loads hoisted above the text normalisation: A/B in the step (rocprof) + head tests
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_model.py > gpurun_out/t76_tests.log 2>&1 || { tail -30 gpurun_out/t76_tests.log; exit 1; }
tail -1 gpurun_out/t76_tests.log
cd /tmp && export TMPDIR=/tmp
for v in new old; do
  if [ $v = old ]; then export EBC_LIB_PATH=$R/clip-ebc_amd/lib/libebc_hip_old.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace -d $R/gpurun_out/t76_$v -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/t76_$v.log 2>&1 || exit 1
done
echo ok
