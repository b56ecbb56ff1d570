#!/bin/bash
# small-channel conv rewrite: its GPU tests on B, then PINN + sampler A/B of lib builds.
mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/b-pinn-kalman-filter_amd/lib
BPK_LIB=$L/libbpk_B.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_pinn.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_small.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_small.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_small.log | head; exit $rc; }
bash tools/gpu_pinn_lib_ab.sh
