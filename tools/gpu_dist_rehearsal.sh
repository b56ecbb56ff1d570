#!/bin/bash
# N=2 rehearsal of the whole bench on one GPU (two ranks share the device; gloo instead of
# RCCL, which cannot put two ranks on one GPU): every phase's distributed path runs.
mkdir -p gpurun_out; export TMPDIR=/tmp
BPK_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 1 --train-steps 2 --cifar-steps 2 --pinn-steps 2 --dps-steps 1 > gpurun_out/bench_n2.log 2> gpurun_out/bench_n2.err || { tail -30 gpurun_out/bench_n2.err; exit 1; }
cat gpurun_out/bench_n2.log
python tools/show_line.py gpurun_out/bench_n2.log; grep -o "\"pinn_losses\": \[[^]]*\]" gpurun_out/bench_n2.log
