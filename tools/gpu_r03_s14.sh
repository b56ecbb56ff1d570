#!/bin/bash
# r03 session 2: 1x1 GEMM epilogue (bias loads batched, straight-line stores for whole tiles)
# and the 8-cin Winograd store_tile skip batching -- GEMM / conv parity tests, then the GEMM
# shapes and the PRE-conv mix on the base vs the new library (same box)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -q -k "conv1x1 or gemm or attention or wino or conv3x3 or resblock" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s14_test.log 2>&1; rc=$?
tail -2 gpurun_out/s14_test.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/s14_test.log | head; exit $rc; }
L=b-pinn-kalman-filter_amd/lib
for v in base new; do
  lib=$L/libbpk.so; [ $v = base ] && lib=$L/libbpk_base.so
  echo "== $v"
  BPK_LIB=$PWD/$lib timeout -k 10 300 python tools/bench_gemm.py 2>/dev/null | python -c "import sys,json;[print(json.loads(l)['shape'], json.loads(l)['gemm_ms'], json.loads(l)['gemm_tflops']) for l in sys.stdin if l.startswith('{')]" || exit 1
done
