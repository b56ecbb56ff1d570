#!/bin/bash
# Round 6 (session 2): deferred two-source weight gradients -- parity tests, the PINN graph
# step at B=8 / B=64 with BPK_DEFER_WGRAD=0 / 1, the aten launch census at B=8.
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "two_sources or deferred or igemm or wgrad" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread -k "pinn" > $O/tests_pinn.log 2>&1 || { tail -30 $O/tests_pinn.log; exit 1; }
tail -2 $O/tests_pinn.log
for d in 0 1; do
  BPK_DEFER_WGRAD=$d timeout -k 10 300 python3 tools/prof_pinn.py graph 8 30 > $O/b8_d$d.log 2>&1 || { tail -20 $O/b8_d$d.log; exit 1; }
  echo "defer $d B=8: $(tail -1 $O/b8_d$d.log | cut -c1-160)"
done
for d in 0 1; do
  BPK_DEFER_WGRAD=$d timeout -k 10 300 python3 tools/prof_pinn.py graph 1 20 > $O/b64_d$d.log 2>&1 || { tail -20 $O/b64_d$d.log; exit 1; }
  echo "defer $d B=64: $(tail -1 $O/b64_d$d.log | cut -c1-160)"
done
timeout -k 10 300 python3 tools/pinn_op_sources.py 8 > $O/aten_sources_b8.txt 2>&1 || { tail -20 $O/aten_sources_b8.txt; exit 1; }
head -3 $O/aten_sources_b8.txt
