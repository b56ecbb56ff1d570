#!/bin/bash
# PINN graph step kernel traces on the final tree (per-step counts from the FilterBatch period)
set -o pipefail
O=gpurun_out/r06profp; mkdir -p $O; export TMPDIR=/tmp; export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
for n in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$n -o pinn --output-format csv -- python3 tools/prof_pinn.py graph $n 5 > $O/p$n.log 2>&1 || { tail -5 $O/p$n.log; exit 1; }
  python3 tools/trace_steps.py $O/p$n/pinn_kernel_trace.csv 5 45 > $O/p${n}_per_step.txt
  head -2 $O/p${n}_per_step.txt
  rm -f $O/p$n/pinn_kernel_trace.csv
done
