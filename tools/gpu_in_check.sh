#!/bin/bash
# fused InstanceNorm+ELU: op tests, PINN parity tests, then PINN bench eager / graph / aten-IN.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_pinn.py tests/test_gpu_configs.py -m gpu -q -k "instance or pinn" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_in.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_in.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-train --no-dps --ns-steps 0 --ncddpmpp-steps 0 --steps 1 --warmup 1 --cifar-steps 0 --pinn-steps 20"
for v in "eager" "graph --pinn-graph" "aten_in BPK_IN_FUSED=0"; do
  set -- $v; name=$1; shift
  flags=""; envs=""
  for a in "$@"; do case $a in --*) flags="$flags $a";; *) envs="$envs $a";; esac; done
  env $envs timeout -k 10 400 python bench.py $B $flags > gpurun_out/pinn_$name.log 2> gpurun_out/pinn_$name.err || { tail -20 gpurun_out/pinn_$name.err; exit 1; }
  echo "$name $(grep -o '"pinn_train_steps_per_s": [0-9.]*' gpurun_out/pinn_$name.log)"
done
