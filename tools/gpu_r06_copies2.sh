#!/bin/bash
# Round 6 (session 2): residual copies 2 vs 4 at the per-rank batches of the 8- and 4-GPU
# points on the final tree, interleaved x3.
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
  for c in 4 2; do
    for n in ${NS:-8 4}; do
      BPK_PINN_COPIES=$c timeout -k 10 300 python3 tools/prof_pinn.py graph $n 30 > $O/n${n}_c${c}_$r.log 2>&1 || { tail -20 $O/n${n}_c${c}_$r.log; exit 1; }
      python3 -c "
import ast; d=ast.literal_eval(open('$O/n${n}_c${c}_$r.log').read().strip().splitlines()[-1]); print('per-rank-of $n copies $c run $r', d['pinn_train_steps_per_s'])"
    done
  done
done
