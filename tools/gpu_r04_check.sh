#!/bin/bash
# Round 4 check: GPU parity tests of the touched kernels (-k filter in $1), then the bench at
# the per-rank batch of the 8-GPU strong-scaled point (global batch 8) and the N=1 sampler at
# B = 64 (no train / PINN / DPS phases), each under its own limit.
mkdir -p gpurun_out; export TMPDIR=/tmp
k=${1:-"upfirdn or conv3x3 or wgrad or attention or conv1x1 or gemm"}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$k" > gpurun_out/t_ops.log 2>&1 || { tail -40 gpurun_out/t_ops.log; exit 1; }
tail -2 gpurun_out/t_ops.log
common="--no-cpu-baseline --no-dps --ns-steps 0 --cifar-steps 0 --no-pinn"
timeout -k 10 400 python bench.py --global-batch 8 --steps 40 $common ${B8_EXTRA:-} > gpurun_out/b8.log 2> gpurun_out/b8.err || { tail -20 gpurun_out/b8.err; exit 1; }
cat gpurun_out/b8.log
timeout -k 10 300 python bench.py --steps 10 --no-train --ncddpmpp-steps 0 $common > gpurun_out/b64.log 2> gpurun_out/b64.err || { tail -20 gpurun_out/b64.err; exit 1; }
cat gpurun_out/b64.log
