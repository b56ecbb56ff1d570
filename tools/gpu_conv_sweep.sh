#!/bin/bash
# Winograd conv sweeps: persistent (default) vs BPK_WINO_PERSIST=0, NCSN++ shapes, conv tests.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_conv_sweep.py > gpurun_out/sweep.log 2>&1 || { cat gpurun_out/sweep.log; exit 1; }
cat gpurun_out/sweep.log
BPK_WINO_PERSIST=0 timeout -k 10 300 python tools/bench_conv_sweep.py > gpurun_out/sweep0.log 2>&1 || { cat gpurun_out/sweep0.log; exit 1; }
echo "== PERSIST=0"; cat gpurun_out/sweep0.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k conv3x3 -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_conv.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_conv.log; exit $rc
