#!/bin/bash
# Round 4: the captured PINN step replayed with fixed parameters (tools/diag_pinn_graph_iso.py).
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARIANTS:-plain churn}; do
  timeout -k 10 300 python tools/diag_pinn_graph_iso.py $v > gpurun_out/pinniso_$v.log 2>&1 || { tail -5 gpurun_out/pinniso_$v.log; exit 1; }
  grep "^${v%%-*}" gpurun_out/pinniso_$v.log | tail -4
done
