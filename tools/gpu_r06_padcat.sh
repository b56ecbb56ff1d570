#!/bin/bash
# Round 6 (session 2): split backward as one zero fill + copies -- parity tests, PINN graph step
# timings by residual copies at B=8 / B=64, kernel trace at B=8.
set -o pipefail
O=gpurun_out/r06g; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "pinn or spatial or channel or split or cat" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in 4 2; do
  BPK_PINN_COPIES=$c timeout -k 10 300 python3 tools/prof_pinn.py graph 8 30 > $O/b8_c$c.log 2>&1 || { tail -20 $O/b8_c$c.log; exit 1; }
done
for c in 2 1; do
  BPK_PINN_COPIES=$c timeout -k 10 300 python3 tools/prof_pinn.py graph 1 20 > $O/b64_c$c.log 2>&1 || { tail -20 $O/b64_c$c.log; exit 1; }
done
for f in b8_c4 b8_c2 b64_c2 b64_c1; do python3 -c "
import ast
d=ast.literal_eval(open('$O/$f.log').read().strip().splitlines()[-1]); print('$f', d['pinn_train_steps_per_s'], d['pinn_losses'])"; done
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p8 -o pinn --output-format csv -- python3 tools/prof_pinn.py graph 8 5 > $O/p8.log 2>&1 || { tail -5 $O/p8.log; exit 1; }
python3 tools/trace_steps.py $O/p8/pinn_kernel_trace.csv 5 45 > $O/p8_per_step.txt
head -24 $O/p8_per_step.txt
rm -f $O/p8/pinn_kernel_trace.csv
