#!/bin/bash
# Round 5: eval-mode-only GroupNorm+SiLU conv fusion under autograd (block test + DPS config
# fixture), the bench line without CPU baselines, and the PINN step's aten-op call sites.
mkdir -p gpurun_out/r05i; export TMPDIR=/tmp
O=gpurun_out/r05i
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "gn_silu_conv_under_autograd or dps_256 or igemm_fwd_dgrad" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --steps 2 --warmup 1 > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log
timeout -k 10 300 python tools/pinn_op_sources.py > $O/pinn_ops.log 2>&1 || { tail -20 $O/pinn_ops.log; exit 1; }
grep -A40 "by call site" $O/pinn_ops.log
