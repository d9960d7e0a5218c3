set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for sd in 0 1; do
  EBC_DEC_SIDE=$sd timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/t23_b.log 2>&1 || exit 1
  echo "side=$sd $(tail -1 gpurun_out/t23_b.log | cut -c80-125)"
done; done
