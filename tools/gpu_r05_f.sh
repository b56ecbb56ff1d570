#!/bin/bash
# Round 5: where the tree stands -- the full default bench line (all phases, CPU baselines
# skipped), the per-rank-of-8 line, and the MIOpen-vs-native census of the training steps.
mkdir -p gpurun_out/r05f; export TMPDIR=/tmp
O=gpurun_out/r05f
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log
timeout -k 10 400 python tools/conv_choices.py > $O/choices.log 2>&1 || { tail -20 $O/choices.log; exit 1; }
tail -25 $O/choices.log
timeout -k 10 600 python bench.py --no-cpu-baseline --per-rank-of 8 > $O/bench_b8.log 2> $O/bench_b8.err || { tail -20 $O/bench_b8.err; exit 1; }
python tools/show_line.py $O/bench_b8.log
