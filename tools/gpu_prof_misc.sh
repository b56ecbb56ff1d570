#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cifar -o cifar --output-format csv -- python tools/prof_cifar.py > gpurun_out/prof_cifar.log 2>&1 || { tail gpurun_out/prof_cifar.log; exit 1; }
echo CIFAR_OK
timeout -k 10 600 python tools/prof_pinn_shapes.py > gpurun_out/pinn_shapes.log 2>&1 || { tail gpurun_out/pinn_shapes.log; exit 1; }
echo SHAPES_OK
