#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "conv1x1" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gemm.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_gemm.log | head; exit $rc; }
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/gemm.log 2>&1 || { cat gpurun_out/gemm.log; exit 1; }
grep shape gpurun_out/gemm.log
