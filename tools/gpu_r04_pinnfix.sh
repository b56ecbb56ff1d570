#!/bin/bash
# Round 4: PINN hipGraph step checks -- fixed-parameter replays (plain / churn), then the
# bench's phase sequence and 24 graph steps vs eager.
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in plain churn; do
  timeout -k 10 300 python tools/diag_pinn_graph_iso.py $v > gpurun_out/pinniso_$v.log 2>&1 || { tail -5 gpurun_out/pinniso_$v.log; exit 1; }
  grep "^$v" gpurun_out/pinniso_$v.log | cut -c1-100
done
for v in bench noeager; do
  timeout -k 10 400 python tools/diag_pinn_bench.py $v 24 > gpurun_out/pinndiag2_$v.log 2>&1 || { tail -5 gpurun_out/pinndiag2_$v.log; exit 1; }
  grep "^$v" gpurun_out/pinndiag2_$v.log | cut -c1-70
done
