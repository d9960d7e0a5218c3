set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t1_tests.log 2>&1 ; echo "tests rc=$?" >> gpurun_out/t1_tests.log
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/t1_bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/t1_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/t1_prof.log 2>&1
