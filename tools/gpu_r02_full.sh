#!/bin/bash
# Full GPU check: all -m gpu tests (parity errors on record), default N=1 bench, smoke().
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench.sh noprof || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" || exit 1
