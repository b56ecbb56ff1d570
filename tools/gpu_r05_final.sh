#!/bin/bash
# Round 5 final lines: the driver's default bench command on the committed tree, then the
# per-rank work of the 8-GPU point (--per-rank-of 8).
mkdir -p gpurun_out/r05final; export TMPDIR=/tmp
O=gpurun_out/r05final
timeout -k 10 900 python bench.py > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log
timeout -k 10 600 python bench.py --per-rank-of 8 --no-cpu-baseline > $O/bench_b8.log 2> $O/bench_b8.err || { tail -20 $O/bench_b8.err; exit 1; }
python tools/show_line.py $O/bench_b8.log
