# r01: GEMM time breakdown (experiment builds: 4 = no epilogue, 6 = no DMA + no epilogue, 1 = no MFMA), glue attribution
set -o pipefail
mkdir -p gpurun_out
for v in base exp4 exp6 exp1 base; do
  if [ $v = base ]; then unset EBC_LIB_PATH; else export EBC_LIB_PATH=clip-ebc_amd/lib/$v/libebc_hip.so; fi
  echo "== $v" >> gpurun_out/t25_gemm.log
  timeout -k 10 120 python tools/gemm_bench.py >> gpurun_out/t25_gemm.log 2>&1 || exit 1
done
unset EBC_LIB_PATH
timeout -k 10 240 python tools/torch_prof.py --steps 3 > gpurun_out/t25_torchprof.log 2>&1
