#!/bin/bash
# Round 4: implicit-GEMM microbench (CIFAR 8^2 shapes, PINN shapes) before the parity tests,
# then tests, census and the training phases (tools/gpu_r04_igemm2.sh).
mkdir -p gpurun_out; export TMPDIR=/tmp
for a in "fwd 128 256 8 8 256 3 1 1" "dgrad 128 256 8 8 256 3 1 1" "fwd 128 512 8 8 256 3 1 1" "dgrad 128 512 8 8 256 3 1 1" "fwd 64 34 32 32 128 3 1 1" "dgrad 64 448 8 8 448 3 1 1" "fwd 64 128 65 65 256 3 2 0"; do
  timeout -k 10 120 python tools/igemm_one.py $a 2>&1 | grep -v amdgpu.ids || exit 1
done
bash tools/gpu_r04_igemm2.sh
