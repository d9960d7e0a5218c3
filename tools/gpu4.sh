# decoder tests + model parity + bench + kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_model.py -v --timeout 120 --timeout-method thread > gpurun_out/t4_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t4_tests.log; exit 1; }
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/t4_bench.log 2>&1 || { tail -30 gpurun_out/t4_bench.log; exit 1; }
tail -1 gpurun_out/t4_bench.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/t4_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/t4_prof.log 2>&1
