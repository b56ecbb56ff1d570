#!/bin/bash
# PINN train step: eager vs hipGraph replay (bench's PINN phase only), same box.
mkdir -p gpurun_out; export TMPDIR=/tmp
B="--no-cpu-baseline --no-train --no-dps --ns-steps 0 --ncddpmpp-steps 0 --steps 1 --warmup 1 --cifar-steps 0 --pinn-steps 20"
timeout -k 10 400 python bench.py $B > gpurun_out/pinn_eager.log 2> gpurun_out/pinn_eager.err || { tail -20 gpurun_out/pinn_eager.err; exit 1; }
grep -o '"pinn_train_steps_per_s": [0-9.]*' gpurun_out/pinn_eager.log
timeout -k 10 400 python bench.py $B --pinn-graph > gpurun_out/pinn_graph.log 2> gpurun_out/pinn_graph.err || { tail -20 gpurun_out/pinn_graph.err; exit 1; }
grep -o '"pinn_train_steps_per_s": [0-9.]*' gpurun_out/pinn_graph.log
