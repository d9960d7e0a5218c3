# r01: crop-split two-stream encoder forward: parity + interleaved A/B bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_model.py > gpurun_out/t27_tests.log 2>&1 || { tail -40 gpurun_out/t27_tests.log; exit 1; }
tail -2 gpurun_out/t27_tests.log
for v in 1 2 1 2; do
  EBC_VIT_STREAMS=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/t27_bench_$v.log 2>&1 || exit 1
  echo "streams=$v $(tail -1 gpurun_out/t27_bench_$v.log | cut -c1-170)"
done
