#!/bin/bash
# Kernel traces of the bench step under two (or more) library builds, same box (lab):
#   tools/lib_trace_ab.sh TAG lib1 lib2 ...   (lib = a directory under clip-ebc_amd/lib, "." = the default build)
# -> gpurun_out/TAG_<lib>/run_results.db (rocprofv3 --kernel-trace), then tools/ab_bench.sh's interleaved bench A/B
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
for l in "$@"; do
  n=$(echo "$l" | tr -c 'a-zA-Z0-9\n' '_')
  export EBC_LIB_PATH=$R/clip-ebc_amd/lib/$l/libebc_hip.so
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_$n -o run -- \
    python3 $R/bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-probe > $R/gpurun_out/${TAG}_$n.log 2>&1) \
    || { tail -20 $R/gpurun_out/${TAG}_$n.log; exit 1; }
  unset EBC_LIB_PATH
done
bash $R/tools/ab_bench.sh $TAG "" "$@"
