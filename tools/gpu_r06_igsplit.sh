#!/bin/bash
# implicit-GEMM split-K target (IGEMM_WANT workgroups per CU for 64x64 tiles, half for the
# others): PINN graph step at B=8 / B=64 per library, interleaved x2
set -o pipefail
O=gpurun_out/r06ig; mkdir -p $O; export TMPDIR=/tmp
L=b-pinn-kalman-filter_amd/lib
for r in 1 2; do
  for v in base w4 w2; do
    lib=$PWD/$L/variants/libbpk_$v.so; [ $v = base ] && lib=$PWD/$L/libbpk.so
    for n in 8 1; do
      BPK_LIB=$lib timeout -k 10 300 python3 tools/prof_pinn.py graph $n 20 > $O/${v}_${n}_$r.log 2>&1 || { tail -20 $O/${v}_${n}_$r.log; exit 1; }
      echo "$v per-rank-of $n run $r: $(grep -o "'pinn_train_steps_per_s': [0-9.]*" $O/${v}_${n}_$r.log)"
    done
  done
done
