#!/bin/bash
# Round 4: PINN losses per step, 12 eager steps vs 12 hipGraph steps from the same fresh state
# and seeds (tools/diag_pinn_bench.py).
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARIANTS:-eager12 noeager}; do
  echo "== $v"
  timeout -k 10 300 python tools/diag_pinn_bench.py $v > gpurun_out/pinndiag_$v.log 2>&1 || { tail -5 gpurun_out/pinndiag_$v.log; exit 1; }
  grep "^$v\|Nan" gpurun_out/pinndiag_$v.log
done
