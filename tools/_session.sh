set -o pipefail
S="gemm:3664,768,3072,2 gemm:3664,768,3072,0 gemm:3664,3072,768,1 gemm:3664,768,768,0"
for v in "" exp1 exp2 exp4 exp6 ""; do
  echo "== lib $v"
  if [ -z "$v" ]; then LP=clip-ebc_amd/lib/libebc_hip.so; else LP=clip-ebc_amd/lib/$v/libebc_hip.so; fi
  EBC_LIB_PATH=$LP timeout -k 10 120 python tools/kbench.py multi $S --reps 50 --rounds 2 || exit 1
done
