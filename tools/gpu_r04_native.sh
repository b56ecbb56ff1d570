#!/bin/bash
# Round 4: native-only conv choices -- the stride-2 igemm vs MIOpen table (split-K workspace cap
# raised), the DSM train + CIFAR + DPS phases at B = 64 on native kernels, and a rocprofv3
# kernel trace of the PINN graph step at B = 64.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_stride2.py > gpurun_out/stride2.log 2>&1 || { tail -20 gpurun_out/stride2.log; exit 1; }
cat gpurun_out/stride2.log
only="--no-cpu-baseline --no-pinn --ns-steps 0 --ncddpmpp-steps 0 --no-roofline"
timeout -k 10 600 python bench.py --steps 3 --warmup 1 $only > gpurun_out/native_train.log 2> gpurun_out/native_train.err || { tail -20 gpurun_out/native_train.err; exit 1; }
python tools/show_line.py gpurun_out/native_train.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04_pinn -o pinn --output-format csv -- python tools/prof_pinn.py > gpurun_out/prof_r04_pinn.log 2>&1 || { tail gpurun_out/prof_r04_pinn.log; exit 1; }
grep "pinn_train_steps" gpurun_out/prof_r04_pinn.log | cut -c1-400
