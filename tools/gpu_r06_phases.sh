#!/bin/bash
# Round 6: PINN graph step split by phase (markers between the derivative passes), B=8 and B=64.
set -o pipefail
O=gpurun_out/r06phases; mkdir -p $O; export TMPDIR=/tmp
for n in 8 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p$n -o ph -- python3 tools/prof_pinn_phases.py $n > $O/p$n.log 2>&1 || { tail -20 $O/p$n.log; exit 1; }
  grep "ms_per_step" $O/p$n.log
  python3 tools/prof_pinn_phases.py --split $O/p$n/ph_kernel_trace.csv | tee $O/p$n.txt
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "higher_order or gn_silu_conv_under" tests/test_gpu_graph.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
