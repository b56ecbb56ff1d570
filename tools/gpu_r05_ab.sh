#!/bin/bash
# Round 5: igemm split-K target sweep on the PINN step (BPK_IGEMM_SPLIT_EXP, timing only).
mkdir -p gpurun_out/r05ab; export TMPDIR=/tmp
O=gpurun_out/r05ab
for e in 0 1 2 3 4 0; do
  export BPK_IGEMM_SPLIT_EXP=$e
  timeout -k 10 300 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-dps --no-train --cifar-steps 0 --steps 1 --warmup 1 > $O/bench_$e.log 2> $O/bench_$e.err || { tail -20 $O/bench_$e.err; exit 1; }
  echo "exp $e: $(python tools/show_line.py $O/bench_$e.log | head -1)"
done
