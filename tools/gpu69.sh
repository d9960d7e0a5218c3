# r01 s5: DDP rehearsal (2 ranks on one GPU, gloo), default bench with CPU baseline, rocprof kernel stats (profile s6: after the GEMM tile retune)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
EBC_BENCH_ONE_DEVICE=1 EBC_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/t69_ddp.log 2>&1 || { tail -30 gpurun_out/t69_ddp.log; exit 1; }
tail -1 gpurun_out/t69_ddp.log | cut -c1-200
timeout -k 10 400 python -u bench.py > gpurun_out/t69_bench.log 2>&1 || { tail -20 gpurun_out/t69_bench.log; exit 1; }
tail -1 gpurun_out/t69_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/t69_prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/t69_prof.log 2>&1 || exit 1
tail -1 $R/gpurun_out/t69_prof.log | cut -c1-200
