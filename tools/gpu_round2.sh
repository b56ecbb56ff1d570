#!/bin/bash
# Full GPU round: parity tests, bench (N=1), rocprofv3 kernel trace of the sampler bench,
# then the Winograd NB=2 variant A/B.  Each GPU step has its own limit; stop at first failure.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --steps 5 --warmup 2 --no-train --no-cpu-baseline --no-pinn --no-dps > gpurun_out/prof.log 2>&1 || exit 1
echo PROF_OK
BPK_WINO_PIPE=2 timeout -k 10 300 python tools/bench_conv.py > gpurun_out/conv_pipe2.log 2>&1 || exit 1
cat gpurun_out/conv_pipe2.log
