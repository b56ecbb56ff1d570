#!/bin/bash
# Round 4 final lines: the default N=1 bench (with the committed PMC traffic) and the per-rank
# rehearsal of the 8-GPU point, each under its own limit.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/bench_final.log 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
python tools/show_line.py gpurun_out/bench_final.log
timeout -k 10 700 python bench.py --per-rank-of 8 --no-cpu-baseline --steps 40 > gpurun_out/rehearse8.log 2> gpurun_out/rehearse8.err || { tail -20 gpurun_out/rehearse8.err; exit 1; }
python tools/show_line.py gpurun_out/rehearse8.log
