#!/bin/bash
# Round 4: the PINN graph diagnostic, then every bench phase at the per-rank batch of the
# strong-scaled 8-GPU run on this one GPU (bench.py --per-rank-of 8).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/diag_pinn_graph.py 64 > gpurun_out/diag_pinn.log 2>&1 || { tail -30 gpurun_out/diag_pinn.log; exit 1; }
grep -v Warn gpurun_out/diag_pinn.log | tail -12
timeout -k 10 700 python bench.py --per-rank-of 8 --no-cpu-baseline --steps 40 > gpurun_out/rehearse8.log 2> gpurun_out/rehearse8.err || { tail -20 gpurun_out/rehearse8.err; exit 1; }
python tools/show_line.py gpurun_out/rehearse8.log
