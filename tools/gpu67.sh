# r01 s5: full GPU suite after the GEMM tile retune + smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t67_tests.log 2>&1 || { tail -40 gpurun_out/t67_tests.log; exit 1; }
tail -1 gpurun_out/t67_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t67_smoke.log 2>&1 || { tail -20 gpurun_out/t67_smoke.log; exit 1; }
tail -1 gpurun_out/t67_smoke.log
