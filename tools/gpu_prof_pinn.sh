#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pinn -o pinn --output-format csv -- python tools/prof_pinn.py > gpurun_out/prof_pinn.log 2>&1 || { tail gpurun_out/prof_pinn.log; exit 1; }
echo PINN_OK
