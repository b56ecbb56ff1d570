#!/bin/bash
# Round 5: graph tests (PINN step with eval steps / reductions between replays at B = 64, PC
# sampler graph with eager work between steps, sharded graph vs eager), the pair-form Winograd
# tests, then a bench line of the sampler + DSM + CIFAR phases.
mkdir -p gpurun_out/r05c; export TMPDIR=/tmp
O=gpurun_out/r05c
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_dist.py tests/test_gpu_ops.py -x -v --timeout 300 --timeout-method thread -k "graph or pair_form or weight_gradient or sharded_pinn or native_leaky" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -40
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pinn --no-dps --ns-steps 0 --ncddpmpp-steps 0 --train-steps 4 --cifar-steps 8 > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log
