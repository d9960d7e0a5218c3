# r01 s5: re-entry validation after container re-creation: full GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t50_tests.log 2>&1 || { tail -40 gpurun_out/t50_tests.log; exit 1; }
tail -1 gpurun_out/t50_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t50_smoke.log 2>&1 || { tail -20 gpurun_out/t50_smoke.log; exit 1; }
tail -1 gpurun_out/t50_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/t50_bench.log 2>&1 || { tail -20 gpurun_out/t50_bench.log; exit 1; }
tail -1 gpurun_out/t50_bench.log
