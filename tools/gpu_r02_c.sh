#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_pinn.py tests/test_abi.py -q -k "grid_sample or dynamics or stencil or abi or export" --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_c.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_c.log; exit $rc
