#!/bin/bash
# Round-2 first GPU call: parity tests, default N=1 bench with the MIOpen cache returned
# under gpurun_out/.  Each GPU step has its own limit; stop at the first failure.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench.sh noprof || exit 1
