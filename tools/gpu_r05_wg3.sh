#!/bin/bash
# Round 5: Winograd weight gradient with range-checked patch loads and buffer-loaded gradient tiles --
# wgrad / GN-conv / train-config tests, wgrad kernel time, DSM + CIFAR phases, and a kernel
# trace of the per-rank B=8 DSM step.
mkdir -p gpurun_out/r05wg3; export TMPDIR=/tmp
O=gpurun_out/r05wg3
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "weight_gradient or gn_silu or wgrad or pair or cifar or train" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o wg --output-format csv -- python3 tools/prof_r02.py wgrad_one > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-dps --no-pinn --steps 1 --warmup 1 > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log | head -1
echo done
