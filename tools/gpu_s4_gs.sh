#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_pinn.py -m gpu -x -q -k "grid_sample or pinn or dispatcher" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gs.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-train --no-dps --ns-steps 0 --ncddpmpp-steps 0 --steps 2 --warmup 1 --cifar-steps 0 > gpurun_out/bench_gs.log 2> gpurun_out/bench_gs.err || { tail -20 gpurun_out/bench_gs.err; exit 1; }
grep -o '"pinn_train_steps_per_s": [0-9.]*' gpurun_out/bench_gs.log
timeout -k 10 300 python -u tools/prof_pinn_ops.py > gpurun_out/pinn_ops.txt 2> gpurun_out/pinn_ops.err || { tail gpurun_out/pinn_ops.err; exit 1; }
echo OPS_OK
