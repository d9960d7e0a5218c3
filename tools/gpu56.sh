# r01 s5: loss parity + A/B (full rows <= 582 points, compact rows <= 1202) vs the previous kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_loss.py > gpurun_out/t56_tests.log 2>&1 || { tail -40 gpurun_out/t56_tests.log; exit 1; }
tail -1 gpurun_out/t56_tests.log
for v in new old; do
  if [ $v = old ]; then export EBC_LIB_PATH=$GRAFT_REPO_ROOT/clip-ebc_amd/lib/libebc_hip_old.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/t56_$v -o run -- python3 tools/loss_ab.py run > gpurun_out/t56_$v.log 2>&1 || { tail -20 gpurun_out/t56_$v.log; exit 1; }
  echo "== $v"; python3 tools/loss_ab.py parse $(find gpurun_out/t56_$v -name "*.db" | head -1)
done
