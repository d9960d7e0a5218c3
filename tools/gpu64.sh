# r01 s5: A/B of the step: 128x96 S3 tiles for the N = 768, K = 768 products (new) vs 128x64 (old), interleaved
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then L=$GRAFT_REPO_ROOT/clip-ebc_amd/lib/libebc_hip_old.so; else L=$GRAFT_REPO_ROOT/clip-ebc_amd/lib/libebc_hip.so; fi
    EBC_LIB_PATH=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/t64_${v}_$r.log 2>&1 || { tail -20 gpurun_out/t64_${v}_$r.log; exit 1; }
    echo "$v $r $(tail -1 gpurun_out/t64_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
