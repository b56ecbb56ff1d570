#!/bin/bash
# full GPU parity tests, then the sampler A/B (tools/gpu_ab_bench.sh $1) on the same box
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
bash tools/gpu_ab_bench.sh $1
