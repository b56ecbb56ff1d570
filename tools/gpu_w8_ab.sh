#!/bin/bash
# 8-wave Winograd workgroup (BPK_WINO_W8=1): conv parity tests with it on, then the per-workgroup
# timeline of the default vs the 8-wave form on the NCSN++ shapes, interleaved.
mkdir -p gpurun_out; export TMPDIR=/tmp
BPK_WINO_W8=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -k "conv3x3 or wino" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/w8_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/w8_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in 0 1; do
  echo "### W8=$v"
  BPK_WINO_W8=$v timeout -k 10 100 python tools/wino_timing.py 128 128 128 256 256 128 256 256 64 512 256 64 256 256 32 > gpurun_out/w8_t.txt 2>&1 || { tail -5 gpurun_out/w8_t.txt; exit 1; }
  grep "==\|  loop\|  prologue \|  epilogue" gpurun_out/w8_t.txt
done; done
