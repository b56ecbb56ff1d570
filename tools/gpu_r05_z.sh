#!/bin/bash
# Round 5: swap_scale in the channels-last layout, grid_sample grad2 with NULL (all-zero)
# incoming gradients -- swap_scale / grid_sample / PINN / graph tests, PINN bench, kernel count.
mkdir -p gpurun_out/r05z; export TMPDIR=/tmp
O=gpurun_out/r05z
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "swap_scale or grid_sample or double_backward" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_pinn.py tests/test_gpu_graph.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "pinn or graph" > $O/pytest2.log 2>&1 || { tail -40 $O/pytest2.log; exit 1; }
tail -1 $O/pytest2.log
timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-dps --no-train --cifar-steps 0 --steps 1 --warmup 1 > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log | head -1
timeout -k 10 400 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-train --no-dps --cifar-steps 0 --steps 1 --warmup 1 --per-rank-of 8 > $O/bench8.log 2> $O/bench8.err || { tail -20 $O/bench8.err; exit 1; }
python tools/show_line.py $O/bench8.log | head -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pinn64 -o pinn --output-format csv -- python3 tools/prof_pinn.py > $O/pinn64.log 2>&1 || { tail -5 $O/pinn64.log; exit 1; }
python tools/trace_steps.py $O/pinn64/pinn_kernel_trace.csv 7 12
