# r01: per-crop / shallow VPT gradient tests, full GPU suite, bench with CPU baseline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t43_tests.log 2>&1 || { tail -40 gpurun_out/t43_tests.log; exit 1; }
tail -1 gpurun_out/t43_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/t43_bench.log 2>&1 || exit 1
tail -1 gpurun_out/t43_bench.log | cut -c1-300
