#!/bin/bash
# Round 5: run-to-run check of the default bench line (all phases in one process) against the
# CIFAR / PINN phases run alone.
mkdir -p gpurun_out/r05ac; export TMPDIR=/tmp
O=gpurun_out/r05ac
timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-dps --no-train --steps 1 --warmup 1 > $O/alone.log 2> $O/alone.err || { tail -20 $O/alone.err; exit 1; }
python tools/show_line.py $O/alone.log | head -1
timeout -k 10 900 python bench.py > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log | head -1
