# r01 s5: 4-rank DDP rehearsal on one MI355X (gloo): the N=4 weak-scaling path end to end
set -o pipefail
mkdir -p gpurun_out
EBC_BENCH_ONE_DEVICE=1 EBC_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/t84_ddp4.log 2>&1 || { tail -30 gpurun_out/t84_ddp4.log; exit 1; }
tail -1 gpurun_out/t84_ddp4.log | cut -c1-300
