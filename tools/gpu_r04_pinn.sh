#!/bin/bash
# Round 4: new-kernel tests (strided GEMM, native Linear / attention autograd), the PINN
# hipGraph-vs-eager test, then the PINN phase of the bench (graph, then eager) at B = 64.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_pinn.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "gemm_sb or linear or attention or conv1x1 or graph" > gpurun_out/t_pinn.log 2>&1 || { tail -40 gpurun_out/t_pinn.log; exit 1; }
tail -2 gpurun_out/t_pinn.log
common="--no-cpu-baseline --no-dps --ns-steps 0 --cifar-steps 0 --no-train --ncddpmpp-steps 0 --no-roofline --steps 2 --warmup 1"
timeout -k 10 400 python bench.py $common > gpurun_out/pinn_graph.log 2> gpurun_out/pinn_graph.err || { tail -20 gpurun_out/pinn_graph.err; exit 1; }
timeout -k 10 400 python bench.py $common --pinn-eager > gpurun_out/pinn_eager.log 2> gpurun_out/pinn_eager.err || { tail -20 gpurun_out/pinn_eager.err; exit 1; }
timeout -k 10 400 python bench.py $common --global-batch 8 > gpurun_out/pinn_graph_b8.log 2> gpurun_out/pinn_graph_b8.err || { tail -20 gpurun_out/pinn_graph_b8.err; exit 1; }
python tools/show_line.py gpurun_out/pinn_graph.log gpurun_out/pinn_eager.log gpurun_out/pinn_graph_b8.log
