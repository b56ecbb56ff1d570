#!/bin/bash
# fused Adam: GPU tests of training paths, then train/CIFAR/PINN bench A (BPK_ADAM_FUSED=0) vs B twice.
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_adam.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_adam.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_adam.log | head -20; exit $rc; }
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then E="BPK_ADAM_FUSED=0"; else E="BPK_ADAM_FUSED=1"; fi
    env $E timeout -k 10 400 python bench.py --steps 5 --train-steps 6 --no-dps --no-cpu-baseline > gpurun_out/abad$v$i.log 2> gpurun_out/abad$v$i.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/abad$v$i.log'));print('$v', d['value'], d.get('train_steps_per_s'), d.get('cifar_train_steps_per_s'), d.get('pinn_train_steps_per_s'))"
  done
done
