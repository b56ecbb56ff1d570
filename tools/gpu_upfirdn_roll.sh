#!/bin/bash
# upfirdn2d rolling kernel: GPU parity tests (automatic strip heights; "$TESTENV" extra env),
# then the A/B ("$@" = variants VAR=VALUE,...)
mkdir -p gpurun_out; export TMPDIR=/tmp
for e in "" $TESTENV; do
  env $e timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "upfirdn or fir or up_or_down" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/roll_test.log 2>&1; rc=$?; echo "tests [$e]: $(tail -1 gpurun_out/roll_test.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/roll_test.log | head; exit $rc; }
done
bash tools/gpu_upfirdn_ab.sh "$@"
