#!/bin/bash
# conv + PINN parity tests, then the PINN bench phase only.
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_pinn.py -k "conv3x3 or pinn or prelim or flownet or pressure" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pinn.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_pinn.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_pinn.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-train --no-dps --no-cpu-baseline > gpurun_out/bench_pinn.log 2> gpurun_out/bench_pinn.err || { tail gpurun_out/bench_pinn.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_pinn.log'));print('pinn', d['pinn_train_steps_per_s'], d['pinn_losses'])"
