#!/bin/bash
# Same-box A/B of two builds of libbpk.so (lib/libbpk_A.so vs lib/libbpk_B.so): conv tests on
# B, conv sweep and sampler bench alternating A / B.
mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/b-pinn-kalman-filter_amd/lib
BPK_LIB=$L/libbpk_B.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "conv3x3" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_ab.log | head; exit $rc; }
for v in A B; do
  BPK_LIB=$L/libbpk_$v.so timeout -k 10 300 python tools/bench_conv_sweep.py > gpurun_out/sweep_$v.log 2>&1 || exit 1
  echo "== $v"; grep cin gpurun_out/sweep_$v.log
done
for i in 1 2; do for v in A B; do
  BPK_LIB=$L/libbpk_$v.so timeout -k 10 300 python bench.py --steps 20 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/ab_$v$i.log 2> gpurun_out/ab_$v$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$v$i.log'));print('$v', d['value'], d['roofline']['ms_per_launch'])"
done; done
