#!/bin/bash
# rocprofv3 kernel traces of the DSM train step (128^2) and the CIFAR-10 train step.
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o train --output-format csv -- python tools/prof_train.py > gpurun_out/prof_train.log 2>&1 || { tail gpurun_out/prof_train.log; exit 1; }
echo TRAIN_OK
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cifar -o cifar --output-format csv -- python tools/prof_cifar.py > gpurun_out/prof_cifar.log 2>&1 || { tail gpurun_out/prof_cifar.log; exit 1; }
echo CIFAR_OK
