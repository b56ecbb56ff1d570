#!/bin/bash
# Round 5: native 2x2 block sum for the ddpm Upsample's input gradient -- sum2x2 / up2 / DPS
# fixture tests, DPS phase.
mkdir -p gpurun_out/r05s2; export TMPDIR=/tmp
O=gpurun_out/r05s2
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "sum2x2 or up2 or dps" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-train --no-pinn --cifar-steps 0 --steps 1 --warmup 1 > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log | head -1
