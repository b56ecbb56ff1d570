#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python tools/prof_pinn_stacks.py > gpurun_out/pinn_stacks.txt 2> gpurun_out/pinn_stacks.err || { tail gpurun_out/pinn_stacks.err; exit 1; }
echo OK
