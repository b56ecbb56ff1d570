#!/bin/bash
# InstanceNorm kernel A/B: op tests on the new library, then the PINN eager step with the
# base / new libraries interleaved (same box).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -k "instance" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_in.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_in.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-train --no-dps --ns-steps 0 --ncddpmpp-steps 0 --steps 1 --warmup 1 --cifar-steps 0 --pinn-steps 20"
L=$PWD/b-pinn-kalman-filter_amd/lib
for r in 1 2; do
  for v in base new; do
    lib=$L/libbpk.so; [ $v = base ] && lib=$L/libbpk_base.so
    BPK_LIB=$lib timeout -k 10 300 python bench.py $B > gpurun_out/pinn_$v.log 2> gpurun_out/pinn_$v.err || { tail -5 gpurun_out/pinn_$v.err; exit 1; }
    echo "$v $(grep -o '"pinn_train_steps_per_s": [0-9.]*' gpurun_out/pinn_$v.log) $(grep -o '"pinn_losses": [^]]*' gpurun_out/pinn_$v.log)"
  done
done
