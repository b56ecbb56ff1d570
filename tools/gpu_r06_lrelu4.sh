#!/bin/bash
# Round 6 (session 2): float4 LeakyReLU kernel -- parity tests, PINN B=8 timing, kernel trace.
set -o pipefail
O=gpurun_out/r06h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "leaky or fused_bias" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/prof_pinn.py graph 8 30 > $O/b8.log 2>&1 || { tail -20 $O/b8.log; exit 1; }
timeout -k 10 300 python3 tools/prof_pinn.py graph 1 20 > $O/b64.log 2>&1 || { tail -20 $O/b64.log; exit 1; }
for f in b8 b64; do python3 -c "
import ast
d=ast.literal_eval(open('$O/$f.log').read().strip().splitlines()[-1]); print('$f', d['pinn_train_steps_per_s'], d['pinn_losses'])"; done
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p8 -o pinn --output-format csv -- python3 tools/prof_pinn.py graph 8 5 > $O/p8.log 2>&1 || { tail -5 $O/p8.log; exit 1; }
python3 tools/trace_steps.py $O/p8/pinn_kernel_trace.csv 5 45 > $O/p8_per_step.txt
head -12 $O/p8_per_step.txt; grep -i "lrelu\|fused_bias" $O/p8_per_step.txt
rm -f $O/p8/pinn_kernel_trace.csv
