#!/bin/bash
# Round 6 (session 2): 1x1 deferral + InstanceNorm fan-out -- parity tests, PINN B=8 / B=64
# graph step with BPK_IN_FANOUT=0 / 1, per-step kernel trace at B=8.
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "two_sources or deferred or instance_norm or conv1x1 or gemm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread -k "pinn" > $O/tests_pinn.log 2>&1 || { tail -30 $O/tests_pinn.log; exit 1; }
tail -2 $O/tests_pinn.log
for d in 0 1; do
  BPK_IN_FANOUT=$d timeout -k 10 300 python3 tools/prof_pinn.py graph 8 30 > $O/b8_f$d.log 2>&1 || { tail -20 $O/b8_f$d.log; exit 1; }
  BPK_IN_FANOUT=$d timeout -k 10 300 python3 tools/prof_pinn.py graph 1 20 > $O/b64_f$d.log 2>&1 || { tail -20 $O/b64_f$d.log; exit 1; }
done
for f in b8_f0 b8_f1 b64_f0 b64_f1; do python3 -c "
import ast
d=ast.literal_eval(open('$O/$f.log').read().strip().splitlines()[-1]); print('$f', d['pinn_train_steps_per_s'], d['pinn_losses'])"; done
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p8 -o pinn --output-format csv -- python3 tools/prof_pinn.py graph 8 5 > $O/p8.log 2>&1 || { tail -5 $O/p8.log; exit 1; }
python3 tools/trace_steps.py $O/p8/pinn_kernel_trace.csv 5 45 > $O/p8_per_step.txt
head -30 $O/p8_per_step.txt
rm -f $O/p8/pinn_kernel_trace.csv
