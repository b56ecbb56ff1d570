#!/bin/bash
# Round 5: igemm split-K ceiling sweep on the PINN step (BPK_IGEMM_MAX_SPLITS, timing only).
mkdir -p gpurun_out/r05y; export TMPDIR=/tmp
O=gpurun_out/r05y
for cap in 0 1 2 4 8 32; do
  if [ $cap -gt 0 ]; then export BPK_IGEMM_MAX_SPLITS=$cap; else unset BPK_IGEMM_MAX_SPLITS; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-dps --no-train --cifar-steps 0 --steps 1 --warmup 1 > $O/bench_$cap.log 2> $O/bench_$cap.err || { tail -20 $O/bench_$cap.err; exit 1; }
  echo "cap $cap: $(python tools/show_line.py $O/bench_$cap.log | head -1)"
done
