# r01 s5: loss kernel threads per workgroup A/B (1024 current vs 512 vs 256)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1024 512 256; do
  if [ $v != 1024 ]; then export EBC_LIB_PATH=$GRAFT_REPO_ROOT/clip-ebc_amd/lib/libebc_hip_nt$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/t57_$v -o run -- python3 tools/loss_ab.py run > gpurun_out/t57_$v.log 2>&1 || { tail -20 gpurun_out/t57_$v.log; exit 1; }
  echo "== $v"; python3 tools/loss_ab.py parse $(find gpurun_out/t57_$v -name "*.db" | head -1)
done
