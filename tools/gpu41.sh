# r01: DACE/Sinkhorn workgroup of 16 lanes per K^T u block, 4-stage butterfly
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_loss.py tests/test_gpu_model.py > gpurun_out/t41_tests.log 2>&1 || { tail -40 gpurun_out/t41_tests.log; exit 1; }
tail -1 gpurun_out/t41_tests.log
timeout -k 10 200 python tools/loss_prof.py 20 250 > gpurun_out/t41_loss_prof.log 2>&1 || { tail -20 gpurun_out/t41_loss_prof.log; exit 1; }
grep -E "^---|crop 0" gpurun_out/t41_loss_prof.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/t41_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/t41_prof.log 2>&1
