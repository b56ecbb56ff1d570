#!/bin/bash
# hipGraph + autograd replay checks (round 3): the pure-aten minimal
# repro (side-stream warm-up -> replays >= 1 return a wrong bias gradient) and the PressureNet
# block compositions (exact on every replay with the warm-up on the current stream).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/diag_graph_autograd.py > gpurun_out/graph_min.log 2>&1 || { tail -5 gpurun_out/graph_min.log; exit 1; }
grep "bias grad" gpurun_out/graph_min.log
timeout -k 10 300 python -u tools/diag_graph_block.py > gpurun_out/graph_block.log 2>&1 || { tail -5 gpurun_out/graph_block.log; exit 1; }
grep "rel err" gpurun_out/graph_block.log | cut -c1-120
