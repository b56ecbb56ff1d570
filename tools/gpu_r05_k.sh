#!/bin/bash
# Round 5: PINN step after the launch cuts -- aten ops by autograd node, and the igemm-vs-
# MIOpen census (the 16 x 256 weight-gradient tiles on the 16-channel convs).
mkdir -p gpurun_out/r05k; export TMPDIR=/tmp
O=gpurun_out/r05k
timeout -k 10 300 python tools/pinn_op_sources.py > $O/pinn_ops.log 2>&1 || { tail -20 $O/pinn_ops.log; exit 1; }
sed -n 1,50p $O/pinn_ops.log
timeout -k 10 300 python tools/conv_choices.py pinn > $O/choices_pinn.log 2>&1 || { tail -20 $O/choices_pinn.log; exit 1; }
grep "wgrad" $O/choices_pinn.log | head -30
