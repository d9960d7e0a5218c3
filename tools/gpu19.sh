set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t20_tests.log 2>&1 || { tail -30 gpurun_out/t20_tests.log; exit 1; }
tail -1 gpurun_out/t20_tests.log
timeout -k 10 60 python -u tools/attn_bench.py > gpurun_out/t20_attn.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/t20_bench.log 2>&1 || exit 1
tail -1 gpurun_out/t20_bench.log | cut -c1-150
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/t20_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/t20_prof.log 2>&1
