#!/bin/bash
# r03 session 2: 1x1 GEMM per-shape rates (tools/bench_gemm.py) for the tuning decision
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/s5_gemm.log 2>&1 || { tail gpurun_out/s5_gemm.log; exit 1; }
cat gpurun_out/s5_gemm.log
