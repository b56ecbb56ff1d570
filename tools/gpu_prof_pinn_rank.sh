#!/bin/bash
# PINN graph step kernel trace at the per-rank B=8 (per-step counts from the FilterBatch period)
set -o pipefail
O=${1:-gpurun_out/pinn_rank}; mkdir -p $O; export TMPDIR=/tmp; export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p8 -o pinn --output-format csv -- python3 tools/prof_pinn.py graph 8 5 > $O/p8.log 2>&1 || { tail -5 $O/p8.log; exit 1; }
python3 tools/trace_steps.py $O/p8/pinn_kernel_trace.csv 5 45 > $O/p8_per_step.txt
head -60 $O/p8_per_step.txt
rm -f $O/p8/pinn_kernel_trace.csv
