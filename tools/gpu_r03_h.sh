#!/bin/bash
# r03: PINN graph replay vs eager after the bench's sampler phase (same process)
mkdir -p gpurun_out; export TMPDIR=/tmp
for d in none nograph nosampler; do
  DIAG=$d timeout -k 10 300 python -u tools/diag_pinn_graph6.py > gpurun_out/diag6_$d.log 2>&1 || { tail -5 gpurun_out/diag6_$d.log; exit 1; }
  echo "== $d"; grep -v Warning gpurun_out/diag6_$d.log | grep "sampler\|^[0-9]" | grep -v "^  "
done
