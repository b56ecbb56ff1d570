#!/bin/bash
# ResnetBlockDDPM fused inference (models/layers.py, BPK_DDPM_FUSED): the ddpm-net GPU tests,
# then the nc_ddpmpp 128^2 ancestral bench line with the fused blocks off / on (one box).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_configs.py tests/test_gpu_dps.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ddpm.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ddpm.log; [ $rc -eq 0 ] || exit $rc
B="--no-train --no-pinn --no-dps --ns-steps 0 --no-cpu-baseline --steps 1 --warmup 1 --ncddpmpp-steps 10"
for f in 0 1 0 1; do
  BPK_DDPM_FUSED=$f timeout -k 10 300 python bench.py $B > gpurun_out/nd_$f.log 2> gpurun_out/nd_$f.err || { tail -5 gpurun_out/nd_$f.err; exit 1; }
  echo "fused=$f $(grep -o '"ncddpmpp_evals_per_s": [0-9.]*' gpurun_out/nd_$f.log)"
done
