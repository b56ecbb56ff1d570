#!/bin/bash
# Round 4: the training-side phases of the bench (DSM 128^2, CIFAR-10, PINN hipGraph, DPS) at
# their default batches, sampler shortened; one bench process under its own limit.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-roofline > gpurun_out/phases.log 2> gpurun_out/phases.err || { tail -20 gpurun_out/phases.err; exit 1; }
python tools/show_line.py gpurun_out/phases.log
