# r01 s5: A/B of the loss kernel: compact factor rows (new) vs full rows (old library)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in new old; do
  if [ $v = old ]; then export EBC_LIB_PATH=$GRAFT_REPO_ROOT/clip-ebc_amd/lib/libebc_hip_old.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/t55_$v -o run -- python3 tools/loss_ab.py run > gpurun_out/t55_$v.log 2>&1 || { tail -20 gpurun_out/t55_$v.log; exit 1; }
  echo "== $v"; python3 tools/loss_ab.py parse $(find gpurun_out/t55_$v -name "*.db" | head -1)
done
