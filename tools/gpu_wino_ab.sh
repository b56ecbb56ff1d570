#!/bin/bash
# Winograd PRE-kernel A/B: conv parity tests on the new library, then the shape-mix
# microbench alternating base / new libraries (same box, interleaved).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -q -k "conv or wino or gn or group" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_wino.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_wino.log; [ $rc -eq 0 ] || exit $rc
L=b-pinn-kalman-filter_amd/lib
for r in 1 2; do
  for v in base new; do
    lib=$L/libbpk.so; [ $v = base ] && lib=$L/libbpk_base.so
    BPK_LIB=$PWD/$lib timeout -k 10 300 python tools/bench_wino_mix.py > gpurun_out/mix_${v}_$r.log 2>&1 || { tail gpurun_out/mix_${v}_$r.log; exit 1; }
    tail -1 gpurun_out/mix_${v}_$r.log
  done
done
