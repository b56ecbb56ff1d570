#!/bin/bash
# Config-parity GPU tests (+ the model / PINN tests whose helpers moved), errors on record.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_models.py tests/test_gpu_pinn.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_cfg.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_cfg.log | tail -60; exit $rc
