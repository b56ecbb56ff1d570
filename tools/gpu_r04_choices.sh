#!/bin/bash
# Round 4: where MIOpen beats the implicit-GEMM kernels (tools/conv_choices.py) in the DSM,
# CIFAR-10 and PINN train steps, each phase under its own limit.
mkdir -p gpurun_out; export TMPDIR=/tmp
for ph in train cifar pinn; do
  timeout -k 10 400 python tools/conv_choices.py $ph > gpurun_out/choices_$ph.log 2>&1 || { tail -20 gpurun_out/choices_$ph.log; exit 1; }
  grep -v "amdgpu.ids\|Warning\|warn" gpurun_out/choices_$ph.log | head -30
done
