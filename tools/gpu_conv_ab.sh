#!/bin/bash
# Winograd conv A/B: the software-pipelined forward kernel vs the serial one, the Winograd
# weight gradient, then the conv parity tests with both opt-ins.  Each GPU step has its
# own time limit; stop at the first failure.
mkdir -p gpurun_out
export TMPDIR=/tmp
BPK_WINO_PIPE=1 timeout -k 10 300 python tools/bench_conv.py > gpurun_out/conv_pipe.log 2>&1 || { cat gpurun_out/conv_pipe.log; exit 1; }
cat gpurun_out/conv_pipe.log
BPK_WINO_PIPE=0 timeout -k 10 300 python tools/bench_conv.py > gpurun_out/conv_serial.log 2>&1 || exit 1
cat gpurun_out/conv_serial.log
BPK_WINO_PIPE=1 BPK_WINO_WGRAD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "conv3x3" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_conv.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_conv.log; [ $rc -eq 0 ] || exit $rc
BPK_WINO_WGRAD=1 timeout -k 10 300 python tools/bench_wgrad.py > gpurun_out/wgrad.log 2>&1 || { cat gpurun_out/wgrad.log; exit 1; }
cat gpurun_out/wgrad.log
