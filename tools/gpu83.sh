# r01 s5 closing check: full GPU suite, smoke, default bench with CPU baseline
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t83_tests.log 2>&1 || { tail -40 gpurun_out/t83_tests.log; exit 1; }
tail -1 gpurun_out/t83_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t83_smoke.log 2>&1 || { tail -20 gpurun_out/t83_smoke.log; exit 1; }
tail -1 gpurun_out/t83_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/t83_bench.log 2>&1 || { tail -20 gpurun_out/t83_bench.log; exit 1; }
tail -1 gpurun_out/t83_bench.log
echo ok
