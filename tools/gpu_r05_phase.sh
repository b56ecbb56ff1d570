#!/bin/bash
# Round 5: the default bench with an allocator reset before the CIFAR / PINN / DPS phases --
# does the CIFAR phase of a full run now measure what it does alone?
mkdir -p gpurun_out/r05phase; export TMPDIR=/tmp
O=gpurun_out/r05phase
for i in 1 2; do
timeout -k 10 900 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 > $O/full_$i.log 2> $O/full_$i.err || { tail -20 $O/full_$i.err; exit 1; }
python tools/show_line.py $O/full_$i.log | head -1
done
