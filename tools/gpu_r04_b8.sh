#!/bin/bash
# Round 4: parity tests of the kernels touched this round, then the per-rank workload of the
# strong-scaled 8-GPU configs[2] point (B = 64/8 = 8) on one GPU -- bench line at global
# batch 8 -- beside the B = 64 sampler on the same box, then a sampler-only rocprofv3 kernel
# trace at B = 8.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "upfirdn or conv3x3 or wgrad or attention or grid_sample" > gpurun_out/t_ops.log 2>&1 || { tail -30 gpurun_out/t_ops.log; exit 1; }
tail -2 gpurun_out/t_ops.log
common="--no-cpu-baseline --no-dps --ns-steps 0 --cifar-steps 0"
timeout -k 10 400 python bench.py --global-batch 8 --steps 40 $common > gpurun_out/b8.log 2> gpurun_out/b8.err || { tail -20 gpurun_out/b8.err; exit 1; }
cat gpurun_out/b8.log
timeout -k 10 300 python bench.py --steps 10 --no-train --no-pinn --ncddpmpp-steps 0 $common > gpurun_out/b64.log 2> gpurun_out/b64.err || { tail -20 gpurun_out/b64.err; exit 1; }
cat gpurun_out/b64.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b8 -o bench --output-format csv -- python bench.py --global-batch 8 --steps 40 --warmup 2 --no-train --no-pinn --ncddpmpp-steps 0 --no-roofline $common > gpurun_out/prof_b8.log 2>&1 || exit 1
echo PROF_OK
