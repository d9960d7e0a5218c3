# r01 s5 final: full GPU suite, smoke (loss + 2-layer step vs reference fixture), default bench with CPU baseline, profile s7
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t77_tests.log 2>&1 || { tail -40 gpurun_out/t77_tests.log; exit 1; }
tail -1 gpurun_out/t77_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t77_smoke.log 2>&1 || { tail -20 gpurun_out/t77_smoke.log; exit 1; }
tail -1 gpurun_out/t77_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/t77_bench.log 2>&1 || { tail -20 gpurun_out/t77_bench.log; exit 1; }
tail -1 gpurun_out/t77_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/t77_prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/t77_prof.log 2>&1 || exit 1
echo ok
