#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -k grid_sample --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gs.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gs.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench.sh noprof || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" || exit 1
