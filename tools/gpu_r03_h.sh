#!/bin/bash
# r03: PINN graph replay vs eager over 26 steps with toggles (DIAG5)
mkdir -p gpurun_out; export TMPDIR=/tmp
for d5 in var0,noopt var0,sync; do
  DIAG=nosampler DIAG5=$d5 DIAG_STEPS=26 timeout -k 10 300 python -u tools/diag_pinn_graph6.py > gpurun_out/diag6_26_$d5.log 2>&1 || { tail -5 gpurun_out/diag6_26_$d5.log; exit 1; }
  echo "== $d5"; grep -v Warning gpurun_out/diag6_26_$d5.log | grep "^[0-9]" | grep -v "^  "
done
