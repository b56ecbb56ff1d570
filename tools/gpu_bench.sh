#!/bin/bash
# bench (N=1) with the MIOpen kernel cache written under gpurun_out/ (so it comes back and
# can be kept in-tree), then the rocprofv3 kernel trace of the PC-sampler phase ALONE
# (no train / PINN / DPS / ns_step / nc_ddpmpp / roofline / upfirdn2d phases), so per-kernel
# shares of a PC step can be read from it.  Each GPU step has its own limit; stop at the
# first failure.  $1 = noprof: bench only; $2 = a tag for the profile directory.
mkdir -p gpurun_out/miopen_cache/kernels gpurun_out/miopen_cache/db
export TMPDIR=/tmp
if [ -d b-pinn-kalman-filter_amd/miopen_cache ]; then cp -r b-pinn-kalman-filter_amd/miopen_cache/. gpurun_out/miopen_cache/; fi
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/gpurun_out/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_cache/db
timeout -k 10 1000 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.log
[ "$1" = "noprof" ] && exit 0
tag=${2:-sampler}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o bench --output-format csv -- python bench.py --steps 10 --warmup 2 --no-train --no-cpu-baseline --no-pinn --no-dps --ns-steps 0 --ncddpmpp-steps 0 --no-roofline > gpurun_out/prof_$tag.log 2>&1 || exit 1
echo PROF_OK
