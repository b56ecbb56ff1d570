#!/bin/bash
# Round 4: implicit-GEMM parity tests, then the igemm-vs-MIOpen census of the PINN / CIFAR /
# DSM train steps (tools/conv_choices.py), each step under its own limit.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "igemm or general or transpose or small_cout or small_channel" > gpurun_out/t_igemm.log 2>&1 || { tail -30 gpurun_out/t_igemm.log; exit 1; }
tail -1 gpurun_out/t_igemm.log
for ph in ${PHASES:-pinn cifar train}; do
  timeout -k 10 400 python tools/conv_choices.py $ph > gpurun_out/choices_$ph.log 2>&1 || { tail -20 gpurun_out/choices_$ph.log; exit 1; }
  grep -v "amdgpu.ids\|Warn\|warn" gpurun_out/choices_$ph.log | head -16
done
