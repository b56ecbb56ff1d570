#!/bin/bash
# Round 4: captured pieces of the PINN step replayed with eager allocations between replays.
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARIANTS:-fwd res full}; do
  timeout -k 10 300 python tools/diag_pinn_graph_bisect.py $v > gpurun_out/pinnbis_$v.log 2>&1 || { tail -5 gpurun_out/pinnbis_$v.log; exit 1; }
  grep "^$v" gpurun_out/pinnbis_$v.log
done
