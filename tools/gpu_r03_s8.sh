#!/bin/bash
# r03 session 2: kernel breakdown of one DPS function-evaluation step (configs[4], 256^2,
# B=16) -- rocprofv3 kernel trace of tools/prof_steps.py dps, sliced between its markers
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s8_dps -o dps -- python3 tools/prof_steps.py dps > gpurun_out/s8_dps.log 2>&1 || { tail -5 gpurun_out/s8_dps.log; exit 1; }
f=$(find gpurun_out/s8_dps -name "*kernel_trace.csv" | head -1)
python3 tools/kernels_between_markers.py "$f" 40 > gpurun_out/s8_dps_breakdown.txt && cat gpurun_out/s8_dps_breakdown.txt
rm -f "$f"
