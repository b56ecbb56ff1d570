#!/bin/bash
# Round 5: kernel trace of the PC sampler (B=64, 1 timed step) to size the 1x1-GEMM launches.
mkdir -p gpurun_out/r05ad; export TMPDIR=/tmp
O=gpurun_out/r05ad
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/b64 -o b64 --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-train --no-pinn --no-dps --cifar-steps 0 --ns-steps 0 --ncddpmpp-steps 0 --no-roofline > $O/b64.log 2>&1 || { tail -5 $O/b64.log; exit 1; }
echo ok
