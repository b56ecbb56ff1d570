#!/bin/bash
# r03 session 2: whole-plane FIR pad(2,2) kernel -- parity tests, then the upfirdn2d A/B
# (base = the new kernel, BPK_UPFIRDN_FIR_PLANE=0 = the rolling kernel), twice.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "upfirdn or fir" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s4_test.log 2>&1; rc=$?
tail -2 gpurun_out/s4_test.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/s4_test.log | head -20; exit $rc; }
bash tools/gpu_upfirdn_ab.sh BPK_UPFIRDN_FIR_PLANE=0 || exit 1
bash tools/gpu_upfirdn_ab.sh BPK_UPFIRDN_FIR_PLANE=0 || exit 1
