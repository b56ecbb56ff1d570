#!/bin/bash
# $1 = env flag (default on): GPU tests, then PINN + DSM-train bench A ($1=0) vs B ($1=1) twice.
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_flag.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_flag.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_flag.log | head -20; exit $rc; }
for i in 1 2; do for v in 0 1; do
  env $1=$v timeout -k 10 400 python bench.py --steps 3 --train-steps 4 --cifar-steps 4 --no-dps --no-cpu-baseline --pinn-steps 8 > gpurun_out/pf$v$i.log 2> gpurun_out/pf$v$i.err || { tail -5 gpurun_out/pf$v$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/pf$v$i.log'));print('$1=$v', d['pinn_train_steps_per_s'], d['train_steps_per_s'], d['cifar_train_steps_per_s'], d['pinn_losses'])"
done; done
