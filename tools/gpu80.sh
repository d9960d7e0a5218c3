# r01 s5: A/B at 32 crops/GPU: 2-stage 128x96 above one wave of tiles (new) vs 3-stage (old), interleaved
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then L=$GRAFT_REPO_ROOT/clip-ebc_amd/lib/libebc_hip_old.so; else L=$GRAFT_REPO_ROOT/clip-ebc_amd/lib/libebc_hip.so; fi
    EBC_LIB_PATH=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --crops-per-gpu 32 > gpurun_out/t80_${v}_$r.log 2>&1 || { tail -20 gpurun_out/t80_${v}_$r.log; exit 1; }
    echo "$v $r $(tail -1 gpurun_out/t80_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
