#!/bin/bash
# steady-state kernel breakdowns of the PINN (fused InstanceNorm+ELU) and CIFAR train steps
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pinn -o pinn --output-format csv -- python tools/prof_pinn.py > gpurun_out/prof_pinn.log 2>&1 || { tail gpurun_out/prof_pinn.log; exit 1; }
python tools/slice_trace.py gpurun_out/prof_pinn/pinn_kernel_trace.csv gs_grad2 0 2 3 50 > gpurun_out/pinn_steady.txt
rm -f gpurun_out/prof_pinn/pinn_kernel_trace.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cifar -o cifar --output-format csv -- python tools/prof_cifar.py > gpurun_out/prof_cifar.log 2>&1 || { tail gpurun_out/prof_cifar.log; exit 1; }
python tools/slice_trace.py gpurun_out/prof_cifar/cifar_kernel_trace.csv multi_tensor_apply 0 2 3 50 > gpurun_out/cifar_steady.txt
rm -f gpurun_out/prof_cifar/cifar_kernel_trace.csv
head -3 gpurun_out/pinn_steady.txt gpurun_out/cifar_steady.txt
