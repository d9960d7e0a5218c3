# r01 s5: loss kernel duration vs point count (rocprof kernel stats of tools/loss_probe.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/t53_prof -o run -- python3 tools/loss_probe.py > gpurun_out/t53_probe.log 2>&1 || { tail -20 gpurun_out/t53_probe.log; exit 1; }
cat gpurun_out/t53_probe.log | grep -v "^W20\|rocprof" | tail -12
find gpurun_out/t53_prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -8
