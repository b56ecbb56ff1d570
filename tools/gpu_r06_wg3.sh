#!/bin/bash
set -o pipefail
O=gpurun_out/r06wg3; mkdir -p $O; export TMPDIR=/tmp
L=b-pinn-kalman-filter_amd/lib
for r in 1 2; do
  for v in base m4 m8 m16; do
    lib=$PWD/$L/variants/libbpk_$v.so; [ $v = base ] && lib=$PWD/$L/libbpk_base.so
    BPK_LIB=$lib timeout -k 10 300 python3 tools/bench_wgrad3x3.py > $O/${v}_$r.log 2>&1 || { tail $O/${v}_$r.log; exit 1; }
    echo "$v $r: $(tail -1 $O/${v}_$r.log)"
  done
done
