#!/bin/bash
# One GPU session: parity tests, op microbenches, bench (N=1), rocprofv3 kernel trace of the
# sampler bench.  Every GPU step has its own time limit; the script stops at the first failure.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 800 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
echo "PYTEST_RC $?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/bench_ops.py > gpurun_out/ops.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_conv.py > gpurun_out/bench_conv.log 2>&1 || exit 1
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --steps 5 --warmup 2 --no-train --no-cpu-baseline --no-pinn --no-dps > gpurun_out/prof.log 2>&1 || exit 1
echo PROF_OK
