#!/bin/bash
# r03: PINN graph replay vs eager in the bench's setup, with toggles
mkdir -p gpurun_out; export TMPDIR=/tmp
for d in none var0 mask1 block var0,mask1; do
  DIAG=$d timeout -k 10 200 python -u tools/diag_pinn_graph5.py > gpurun_out/diag5_$d.log 2>&1 || { tail -5 gpurun_out/diag5_$d.log; exit 1; }
  grep -v Warning gpurun_out/diag5_$d.log | grep "DIAG\|^[0-9]" | grep -v "^  "
done
