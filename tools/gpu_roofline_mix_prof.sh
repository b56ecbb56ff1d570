#!/bin/bash
# The bench's roofline kernel (Winograd PRE conv over the NCSN++ 128^2 shape mix) two ways on
# one box: HIP events (tools/bench_wino_mix.py, as bench.py) and a rocprofv3 kernel trace of
# the same program; then the kernel-trace stats summary kept for profiles/.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_wino_mix.py > gpurun_out/mix_events.log 2>&1 || { tail -5 gpurun_out/mix_events.log; exit 1; }
tail -1 gpurun_out/mix_events.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mix -o mix --output-format csv -- python tools/bench_wino_mix.py > gpurun_out/mix_prof.log 2>&1 || { tail -5 gpurun_out/mix_prof.log; exit 1; }
tail -1 gpurun_out/mix_prof.log
python tools/roofline_mix_from_trace.py gpurun_out/prof_mix/mix_kernel_trace.csv > gpurun_out/mix_trace.json && cat gpurun_out/mix_trace.json
rm -f gpurun_out/prof_mix/mix_kernel_trace.csv
