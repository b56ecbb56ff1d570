#!/bin/bash
# Round 4: PINN phase of the bench, eager step vs hipGraph step (10 timed steps each, B = 64).
mkdir -p gpurun_out; export TMPDIR=/tmp
only="--steps 2 --warmup 1 --no-cpu-baseline --no-train --cifar-steps 0 --no-dps --ns-steps 0 --ncddpmpp-steps 0 --no-roofline"
timeout -k 10 400 python bench.py $only --pinn-eager > gpurun_out/pinn_eager.log 2> gpurun_out/pinn_eager.err || { tail -20 gpurun_out/pinn_eager.err; exit 1; }
grep -o '"pinn_train_steps_per_s": [0-9.]*\|"pinn_losses": \[[^]]*\]' gpurun_out/pinn_eager.log
timeout -k 10 400 python bench.py $only > gpurun_out/pinn_graph.log 2> gpurun_out/pinn_graph.err || { tail -20 gpurun_out/pinn_graph.err; exit 1; }
grep -o '"pinn_train_steps_per_s": [0-9.]*\|"pinn_losses": \[[^]]*\]' gpurun_out/pinn_graph.log
