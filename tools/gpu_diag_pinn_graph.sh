#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
for e in "obs,copy,nan,ema,static" "static" "obs" "copy,nan,ema"; do
  DIAG_T=$e timeout -k 10 300 python tools/diag_pinn_graph3.py > gpurun_out/diag_pg3.log 2>&1 || { tail -20 gpurun_out/diag_pg3.log; exit 1; }
  echo "== $e"; grep "replay\|eager" gpurun_out/diag_pg3.log | grep -v print | tr '\n' ' ' | sed 's/replay/\nreplay/g' | awk '{print $1,$2,$3}' | tr '\n' ' '; echo
done
