#!/bin/bash
# PINN residual sensitivities vs float64 truth (small and full config).
mkdir -p gpurun_out; export TMPDIR=/tmp
for w in small full; do
  timeout -k 10 240 python tools/diag_pinn_f64.py $w >> gpurun_out/diag_f64.jsonl 2>> gpurun_out/diag_f64.err || exit 1
done
