#!/bin/bash
# PINN step profile: rocprofv3 steady-state kernel slice + torch.profiler op table.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pinn -o pinn --output-format csv -- python tools/prof_pinn.py > gpurun_out/prof_pinn.log 2>&1 || { tail gpurun_out/prof_pinn.log; exit 1; }
python tools/slice_trace.py gpurun_out/prof_pinn/pinn_kernel_trace.csv gs_grad2 0 2 3 60 > gpurun_out/pinn_steady.txt
rm -f gpurun_out/prof_pinn/pinn_kernel_trace.csv
head -3 gpurun_out/pinn_steady.txt
timeout -k 10 400 python tools/prof_pinn_ops.py > gpurun_out/pinn_ops.txt 2> gpurun_out/pinn_ops.err || { tail gpurun_out/pinn_ops.err; exit 1; }
echo OK
