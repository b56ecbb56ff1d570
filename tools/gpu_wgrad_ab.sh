#!/bin/bash
# wgrad parity tests, then the Winograd weight-gradient microbench: pipelined (default) vs
# BPK_WGRAD_PIPE=0, then the train phase of the bench.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "conv3x3" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_conv.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_conv.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_conv.log | head; exit $rc; }
timeout -k 10 300 python tools/bench_wgrad.py > gpurun_out/wgrad_pipe.log 2>&1 || { cat gpurun_out/wgrad_pipe.log; exit 1; }
echo "== pipe"; cat gpurun_out/wgrad_pipe.log
BPK_WGRAD_PIPE=0 timeout -k 10 300 python tools/bench_wgrad.py > gpurun_out/wgrad_serial.log 2>&1 || exit 1
echo "== serial"; cat gpurun_out/wgrad_serial.log
