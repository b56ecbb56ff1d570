#!/bin/bash
# PINN step: MIOpen immediate mode (0) vs find / cudnn.benchmark (1), with a heartbeat.
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
(while true; do sleep 50; echo heartbeat; done) & HB=$!
timeout -k 10 400 python tools/pinn_find.py 0 2>&1 | grep -v Warning; rc=$?
[ $rc -eq 0 ] && { timeout -k 10 600 python tools/pinn_find.py 1 2>&1 | grep -v Warning; rc=$?; }
kill $HB
exit $rc
