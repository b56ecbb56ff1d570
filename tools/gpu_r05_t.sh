#!/bin/bash
# Round 5: DSM train + CIFAR bench phases on the current igemm, and a kernel trace of the
# CIFAR train steps (per-step breakdown of the timed steps).
mkdir -p gpurun_out/r05t; export TMPDIR=/tmp
O=gpurun_out/r05t
timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-dps --no-pinn --steps 1 --warmup 1 > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log | head -1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/cifar -o cifar --output-format csv -- python3 tools/prof_cifar.py > $O/cifar.log 2>&1 || { tail -5 $O/cifar.log; exit 1; }
python tools/trace_steps.py $O/cifar/cifar_kernel_trace.csv 3 45
