# r01 s5: augmentation: op lists spread over row-block workgroups; parity + bench + kernel stats
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_augment.py > gpurun_out/t62_tests.log 2>&1 || { tail -60 gpurun_out/t62_tests.log; exit 1; }
tail -1 gpurun_out/t62_tests.log
timeout -k 10 300 python -u bench.py --augment --steps 20 --warmup 3 > gpurun_out/t62_aug.log 2>&1 || { tail -30 gpurun_out/t62_aug.log; exit 1; }
tail -1 gpurun_out/t62_aug.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/t62_prof -o run -- python3 $R/bench.py --augment --steps 5 --warmup 1 > $R/gpurun_out/t62_prof.log 2>&1 || exit 1
