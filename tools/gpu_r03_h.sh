#!/bin/bash
# r03: PINN graph replay vs eager over 26 steps (bench setup), then the bench's own PINN phase
# in graph mode, and the PINN phase eager with the K16 Winograd form off / on
mkdir -p gpurun_out; export TMPDIR=/tmp
DIAG=nosampler DIAG_STEPS=26 timeout -k 10 300 python -u tools/diag_pinn_graph6.py > gpurun_out/diag6_26.log 2>&1 || { tail -5 gpurun_out/diag6_26.log; exit 1; }
grep -v Warning gpurun_out/diag6_26.log | grep "^[0-9]" | grep -v "^  "
for k in 0 2; do
  BPK_WINO_K16=$k timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-train --no-dps --ns-steps 0 --ncddpmpp-steps 0 --no-roofline --no-cpu-baseline --pinn-steps 10 > gpurun_out/bench_pinn_k$k.log 2> gpurun_out/bench_pinn_k$k.err || { tail -20 gpurun_out/bench_pinn_k$k.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_pinn_k$k.log').read().strip().splitlines()[-1]); print('K16=$k', {k: d[k] for k in ('pinn_train_steps_per_s', 'pinn_losses')})"
done
