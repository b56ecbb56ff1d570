#!/bin/bash
# Round 4: implicit-GEMM + small-channel parity tests, the stride-2 FIR-down table, then the
# igemm census of the DSM and CIFAR-10 train steps.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "igemm or general or transpose or small_cout or small_channel or small_cin or conv3x3 or cifar or pinn" > gpurun_out/t_igemm.log 2>&1 || { tail -30 gpurun_out/t_igemm.log; exit 1; }
tail -1 gpurun_out/t_igemm.log
for ph in train cifar pinn; do
  timeout -k 10 400 python tools/conv_choices.py $ph > gpurun_out/choices_$ph.log 2>&1 || { tail -20 gpurun_out/choices_$ph.log; exit 1; }
  grep -v "amdgpu.ids\|Warn\|warn" gpurun_out/choices_$ph.log | head -8
done
timeout -k 10 700 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-roofline > gpurun_out/phases.log 2> gpurun_out/phases.err || { tail -20 gpurun_out/phases.err; exit 1; }
python tools/show_line.py gpurun_out/phases.log
