#!/bin/bash
# r03 session 2: igemm epilogue (bias batched, straight-line stores for whole tiles) --
# igemm parity tests, then the PINN / CIFAR igemm shape sums on the base vs the new library
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -q -k "igemm or general or conv2d" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s16_test.log 2>&1; rc=$?
tail -2 gpurun_out/s16_test.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/s16_test.log | head; exit $rc; }
L=b-pinn-kalman-filter_amd/lib
for r in 1 2; do for v in base new; do
  lib=$L/libbpk.so; [ $v = base ] && lib=$L/libbpk_base.so
  BPK_LIB=$PWD/$lib timeout -k 10 400 python tools/bench_igemm.py > gpurun_out/s16_ig_${v}_$r.log 2>&1 || { tail gpurun_out/s16_ig_${v}_$r.log; exit 1; }
  echo "$v: $(grep workload gpurun_out/s16_ig_${v}_$r.log | python -c "import sys,json;[print(json.loads(l)['workload'][:10], json.loads(l)['igemm_ms_per_step']) for l in sys.stdin]" | tr '\n' ' ')"
done; done
