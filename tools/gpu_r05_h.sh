#!/bin/bash
# Round 5: GroupNorm+SiLU inside the conv's input load under autograd -- block-level test,
# the config fixtures (DPS 256^2, CIFAR configs, train), the igemm tests (16 x 256 weight-
# gradient tiles), then the bench phases against the unfused path (BPK_GN_CONV_AD=0), and
# the PINN step's aten-op attribution.
mkdir -p gpurun_out/r05h; export TMPDIR=/tmp
O=gpurun_out/r05h
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread -k "gn_silu_conv_under_autograd or dps_256 or cifar_config or train or igemm" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 1 0; do
  BPK_GN_CONV_AD=$v timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --steps 2 --warmup 1 > $O/bench_$v.log 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  echo "gn_conv_ad=$v"; python tools/show_line.py $O/bench_$v.log
done
timeout -k 10 300 python tools/pinn_op_sources.py > $O/pinn_ops.log 2>&1 || { tail -20 $O/pinn_ops.log; exit 1; }
head -40 $O/pinn_ops.log
