#!/bin/bash
# GPU tests on lib B, then DSM / CIFAR / PINN train A/B of lib/libbpk_A.so vs libbpk_B.so.
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
L=$PWD/b-pinn-kalman-filter_amd/lib
BPK_LIB=$L/libbpk_B.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_lt.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_lt.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_lt.log | head; exit $rc; }
for i in 1 2; do for v in A B; do
  BPK_LIB=$L/libbpk_$v.so timeout -k 10 400 python bench.py --steps 3 --train-steps 4 --cifar-steps 6 --no-dps --no-cpu-baseline --pinn-steps 8 > gpurun_out/lt_$v$i.log 2> gpurun_out/lt_$v$i.err || { tail -5 gpurun_out/lt_$v$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/lt_$v$i.log'));print('$v', d['train_steps_per_s'], d['cifar_train_steps_per_s'], d['pinn_train_steps_per_s'], d['train_loss'])"
done; done
