#!/bin/bash
# Round 5: GroupNorm backward's parameter-gradient reductions in one launch -- GN / GN-conv /
# train-config tests, DSM train + CIFAR + DPS bench phases.
mkdir -p gpurun_out/r05v; export TMPDIR=/tmp
O=gpurun_out/r05v
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread -k "group_norm or gn_ or cifar or ddpm or train or dps" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-pinn --steps 1 --warmup 1 > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log | head -1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/cifar -o cifar --output-format csv -- python3 tools/prof_cifar.py > $O/cifar.log 2>&1 || { tail -5 $O/cifar.log; exit 1; }
python tools/trace_steps.py $O/cifar/cifar_kernel_trace.csv 3 30
