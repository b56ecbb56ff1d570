#!/bin/bash
# Round 5: GroupNorm+SiLU inside the conv under autograd for TRAINING (BPK_GN_CONV_AD_TRAIN),
# interleaved A/B of the DSM + CIFAR phases after this round's weight-gradient changes.
mkdir -p gpurun_out/r05gnad; export TMPDIR=/tmp
O=gpurun_out/r05gnad
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "gn_silu_conv" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
for v in 0 1; do
  BPK_GN_CONV_AD_TRAIN=$v timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-dps --no-pinn --steps 1 --warmup 1 --train-steps 8 --cifar-steps 12 > $O/b_${v}_$i.log 2> $O/b_${v}_$i.err || { tail -20 $O/b_${v}_$i.err; exit 1; }
  echo "train_ad=$v run $i: $(python tools/show_line.py $O/b_${v}_$i.log | head -1)"
done
done
