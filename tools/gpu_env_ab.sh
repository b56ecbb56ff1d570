#!/bin/bash
# conv tests under variant B ($1 = env assignment), conv sweep A vs B, sampler bench A/B x2
mkdir -p gpurun_out; export TMPDIR=/tmp
env $1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "conv3x3" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_envab.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_envab.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_envab.log | head; exit $rc; }
timeout -k 10 300 python tools/bench_conv_sweep.py > gpurun_out/sweepA.log 2>&1 || exit 1
env $1 timeout -k 10 300 python tools/bench_conv_sweep.py > gpurun_out/sweepB.log 2>&1 || exit 1
echo "== A"; grep cin gpurun_out/sweepA.log; echo "== B"; grep cin gpurun_out/sweepB.log
bash tools/gpu_ab_bench.sh $1
