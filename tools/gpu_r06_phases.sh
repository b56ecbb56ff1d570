#!/bin/bash
# Round 6: PINN graph step split by phase (markers between the derivative passes) at the
# per-rank B=8 and at B=64 (copies auto), the aten launches' autograd sources at B=8, and the
# graph-step tests.
set -o pipefail
O=gpurun_out/r06phases; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_graph.py tests/test_gpu_configs.py -k "pinn or graph" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for n in 8 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p$n -o ph -- python3 tools/prof_pinn_phases.py $n > $O/p$n.log 2>&1 || { tail -20 $O/p$n.log; exit 1; }
  grep "ms_per_step" $O/p$n.log
  python3 tools/prof_pinn_phases.py --split $O/p$n/ph_kernel_trace.csv | tee $O/p$n.txt
  python3 tools/trace_steps.py $O/p$n/ph_kernel_trace.csv 3 40 > $O/p${n}_per_step.txt || true
done
timeout -k 10 300 python3 tools/step_op_sources.py pinn --per-rank-of 8 > $O/aten_b8.txt 2>&1 || { tail -20 $O/aten_b8.txt; exit 1; }
head -50 $O/aten_b8.txt
