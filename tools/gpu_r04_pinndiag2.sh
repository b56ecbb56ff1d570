#!/bin/bash
# Round 4: PINN losses per step over 24 steps, eager vs hipGraph from a fresh state.
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in eager12 noeager; do
  echo "== $v"
  timeout -k 10 400 python tools/diag_pinn_bench.py $v 24 > gpurun_out/pinndiag2_$v.log 2>&1 || { tail -5 gpurun_out/pinndiag2_$v.log; exit 1; }
  grep "^$v" gpurun_out/pinndiag2_$v.log | cut -c1-120
done
