# r01: 160x256 conv tiles (cfg 40 2-stage / 41 3-stage); LayerNorm 1 row per wave with hoisted loads
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_decoder.py > gpurun_out/t34_tests.log 2>&1 || { tail -40 gpurun_out/t34_tests.log; exit 1; }
tail -1 gpurun_out/t34_tests.log
for v in "" "EBC_CONV_CFG=40" "EBC_CONV_CFG=41" ""; do
  echo "== $v"; env $v timeout -k 10 120 python tools/conv_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
EBC_CONV_CFG=41 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_decoder.py > gpurun_out/t34_tests41.log 2>&1 || { tail -40 gpurun_out/t34_tests41.log; exit 1; }
tail -1 gpurun_out/t34_tests41.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/t34_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/t34_prof.log 2>&1
