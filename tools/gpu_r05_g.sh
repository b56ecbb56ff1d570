#!/bin/bash
# Round 5: kernel mix of the PINN graph step (B=64 and B=8) after the native LeakyReLU, and
# the CIFAR / PINN MIOpen-vs-native census.
mkdir -p gpurun_out/r05g; export TMPDIR=/tmp
O=gpurun_out/r05g
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pinn64 -o pinn --output-format csv -- python3 tools/prof_pinn.py > $O/pinn64.log 2>&1 || { tail -5 $O/pinn64.log; exit 1; }
tail -1 $O/pinn64.log
timeout -k 10 300 python tools/conv_choices.py cifar > $O/choices_cifar.log 2>&1 || { tail -20 $O/choices_cifar.log; exit 1; }
grep -v amdgpu.ids $O/choices_cifar.log | head -20
timeout -k 10 300 python tools/conv_choices.py pinn > $O/choices_pinn.log 2>&1 || { tail -20 $O/choices_pinn.log; exit 1; }
grep -v amdgpu.ids $O/choices_pinn.log | head -20
