#!/bin/bash
# rocprofv3 kernel trace of the PC-sampler bench (graph replay), 10 timed steps.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_samp -o samp --output-format csv -- python bench.py --steps 10 --warmup 2 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/prof_samp.log 2> gpurun_out/prof_samp.err || { tail gpurun_out/prof_samp.err; exit 1; }
cat gpurun_out/prof_samp.log
