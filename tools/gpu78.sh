# r01 s5: config-4 per-rank shape (32 crops/GPU): bench + tile sweep at M = 32*229 = 7328
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --crops-per-gpu 32 --no-cpu-baseline > gpurun_out/t78_bench32.log 2>&1 || { tail -20 gpurun_out/t78_bench32.log; exit 1; }
tail -1 gpurun_out/t78_bench32.log | cut -c1-300
for c in 0 2 3 4 5 13 1 7 10 20; do
  echo "== cfg $c" >> gpurun_out/t78_sweep.log
  GB_M=7328 EBC_GEMM_CFG=$c timeout -k 10 120 python tools/gemm_bench.py >> gpurun_out/t78_sweep.log 2>&1 || { tail -20 gpurun_out/t78_sweep.log; exit 1; }
done
echo done
