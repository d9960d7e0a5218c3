# r01 s5: augmentation bench (row f2) + rocprof kernel stats of it
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --augment --steps 20 --warmup 3 > gpurun_out/t60_aug.log 2>&1 || { tail -30 gpurun_out/t60_aug.log; exit 1; }
tail -1 gpurun_out/t60_aug.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/t60_prof -o run -- python3 $R/bench.py --augment --steps 5 --warmup 1 > $R/gpurun_out/t60_prof.log 2>&1 || exit 1
