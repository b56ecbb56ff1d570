#!/bin/bash
# rocprofv3 kernel trace of the PINN train step (2 warm-up + 3 steps); the steady-state slice
# is computed on the box and the (large) trace deleted so gpurun_out/ stays small.
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pinn -o pinn --output-format csv -- python tools/prof_pinn.py > gpurun_out/prof_pinn.log 2>&1 || { tail gpurun_out/prof_pinn.log; exit 1; }
python tools/slice_trace.py gpurun_out/prof_pinn/pinn_kernel_trace.csv gs_grad2 0 2 3 40 > gpurun_out/pinn_steady.txt
rm -f gpurun_out/prof_pinn/pinn_kernel_trace.csv
echo PINN_OK
