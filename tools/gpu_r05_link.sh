#!/bin/bash
# Round 5: residual-block skip gradient handed to the GroupNorm backward (SkipLink) -- block /
# GN / DPS fixture tests, DPS phase with the link on and off.
mkdir -p gpurun_out/r05link; export TMPDIR=/tmp
O=gpurun_out/r05link
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread -k "skip_link or gn_silu or group_norm or dps or up2" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0 1; do
  BPK_SKIP_LINK=$v timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-train --no-pinn --cifar-steps 0 --steps 1 --warmup 1 --dps-steps 3 > $O/b_$v.log 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  echo "link=$v: $(python tools/show_line.py $O/b_$v.log | head -1)"
done
