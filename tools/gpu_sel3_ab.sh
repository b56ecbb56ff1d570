#!/bin/bash
# small-image 3x3 conv selection (Winograd vs igemm, timed): conv / PINN / config parity tests,
# then the PINN and CIFAR train steps with BPK_CONV3_SELECT=0 / 1 interleaved.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_pinn.py tests/test_gpu_configs.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sel3.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_sel3.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-train --no-dps --ns-steps 0 --ncddpmpp-steps 0 --steps 1 --warmup 1 --pinn-steps 20 --cifar-steps 6"
for r in 1 2; do
  for v in 0 1; do
    BPK_CONV3_SELECT=$v timeout -k 10 400 python bench.py $B > gpurun_out/sel3_$v.log 2> gpurun_out/sel3_$v.err || { tail -5 gpurun_out/sel3_$v.err; exit 1; }
    echo "sel=$v $(grep -o '"pinn_train_steps_per_s": [0-9.]*' gpurun_out/sel3_$v.log) $(grep -o '"cifar_train_steps_per_s": [0-9.]*' gpurun_out/sel3_$v.log) $(grep -o '"pinn_losses": [^]]*' gpurun_out/sel3_$v.log)"
  done
done
