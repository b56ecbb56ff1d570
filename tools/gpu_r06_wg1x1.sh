#!/bin/bash
# 1x1 weight gradient: split rule + unrolled split reduction (tools/bench_wgrad1x1.py), base vs new;
# then the 1x1 / wgrad parity tests and the PINN step at B=8 / B=64 on the new library.
set -o pipefail
O=gpurun_out/r06wg; mkdir -p $O; export TMPDIR=/tmp
L=b-pinn-kalman-filter_amd/lib
for r in 1 2; do
  for v in base new; do
    lib=$PWD/$L/variants/libbpk_$v.so; [ $v = base ] && lib=$PWD/$L/libbpk_base.so
    BPK_LIB=$lib timeout -k 10 300 python3 tools/bench_wgrad1x1.py > $O/f_${v}_$r.log 2>&1 || { tail $O/f_${v}_$r.log; exit 1; }
    echo "$v $r: $(tail -1 $O/f_${v}_$r.log)"
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "1x1 or gemm or wgrad" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for n in 8 1; do
  timeout -k 10 300 python3 tools/prof_pinn.py graph $n 20 > $O/pinn_$n.log 2>&1 || { tail -20 $O/pinn_$n.log; exit 1; }
  echo "pinn per-rank-of $n: $(grep -o "'pinn_train_steps_per_s': [0-9.]*" $O/pinn_$n.log)"
done
