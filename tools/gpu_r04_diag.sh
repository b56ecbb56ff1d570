#!/bin/bash
# Round 4 diagnostics: per-workgroup phase timeline of the Winograd PRE conv (timing build,
# tools/wino_timing.py) on the 128- and 256-input-channel 128^2 shapes and the 32^2 / 16^2
# shapes at B = 8, then the upfirdn2d microbench (x2).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python tools/wino_timing.py 128 128 128 256 256 128 > gpurun_out/wtime.log 2>&1 || { tail -20 gpurun_out/wtime.log; exit 1; }
grep -v amdgpu.ids gpurun_out/wtime.log
for i in 1 2; do timeout -k 10 120 python tools/bench_upfirdn.py 2>&1 | grep -v amdgpu.ids || exit 1; done
