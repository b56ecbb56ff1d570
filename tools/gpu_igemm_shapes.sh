#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "igemm or general or transpose" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ig.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ig.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_igemm.py > gpurun_out/igemm_shapes.jsonl 2> gpurun_out/igemm_shapes.err || { tail -20 gpurun_out/igemm_shapes.err; exit 1; }
cat gpurun_out/igemm_shapes.jsonl
