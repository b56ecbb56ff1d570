#!/bin/bash
# GroupNorm parity tests, then the train-step profile.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "group_norm" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gn.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gn.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_gn.log | head; exit $rc; }
bash tools/gpu_prof_train.sh
