#!/bin/bash
# Round-6 final bench lines on the final tree: the driver's default command (twice) and the
# per-rank work of the 8-GPU point.
set -o pipefail
O=gpurun_out/r06final; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 900 python3 bench.py > $O/bench_$r.json 2> $O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  tail -c 300 $O/bench_$r.json; echo
done
timeout -k 10 900 python3 bench.py --per-rank-of 8 > $O/per_rank_of_8.json 2> $O/per_rank_of_8.err || { tail -20 $O/per_rank_of_8.err; exit 1; }
echo done
