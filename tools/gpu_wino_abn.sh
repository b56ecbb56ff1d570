#!/bin/bash
# Winograd A/B over N library variants: conv parity tests on each non-base variant, then the
# shape-mix microbench interleaved over the variants (same box).  usage: gpu_wino_abn.sh v1 v2 ...
mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/b-pinn-kalman-filter_amd/lib
for v in "$@"; do
  BPK_LIB=$L/libbpk_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -q -k "conv or wino" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_wino_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/pytest_wino_$v.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in base "$@"; do
    BPK_LIB=$L/libbpk_$v.so timeout -k 10 300 python tools/bench_wino_mix.py > gpurun_out/mix_${v}_$r.log 2>&1 || { tail gpurun_out/mix_${v}_$r.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/mix_${v}_$r.log)"
  done
done
