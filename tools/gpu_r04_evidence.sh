#!/bin/bash
# Round 4 evidence on the final tree: rocprofv3 kernel traces (--stats) of the PC-sampler
# phase alone at B = 64 (the N=1 line) and at B = 8 (the 8-GPU point's per-rank work), and of
# the DSM train step at B = 64.  Each step under its own limit; stop at the first failure.
mkdir -p gpurun_out; export TMPDIR=/tmp
only="--no-train --no-cpu-baseline --no-pinn --no-dps --ns-steps 0 --ncddpmpp-steps 0 --no-roofline --cifar-steps 0"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04_b64 -o bench --output-format csv -- python bench.py --steps 10 --warmup 2 $only > gpurun_out/prof_r04_b64.log 2>&1 || { tail gpurun_out/prof_r04_b64.log; exit 1; }
rm -f gpurun_out/prof_r04_*/*_kernel_trace.csv; echo PROF_B64_OK
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04_b8 -o bench --output-format csv -- python bench.py --global-batch 8 --steps 40 --warmup 2 $only > gpurun_out/prof_r04_b8.log 2>&1 || { tail gpurun_out/prof_r04_b8.log; exit 1; }
rm -f gpurun_out/prof_r04_*/*_kernel_trace.csv; echo PROF_B8_OK
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04_train -o train --output-format csv -- python tools/prof_train.py > gpurun_out/prof_r04_train.log 2>&1 || { tail gpurun_out/prof_r04_train.log; exit 1; }
rm -f gpurun_out/prof_r04_*/*_kernel_trace.csv; echo PROF_TRAIN_OK
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04_pinn -o pinn --output-format csv -- python tools/prof_pinn.py > gpurun_out/prof_r04_pinn.log 2>&1 || { tail gpurun_out/prof_r04_pinn.log; exit 1; }
rm -f gpurun_out/prof_r04_*/*_kernel_trace.csv; echo PROF_PINN_OK
