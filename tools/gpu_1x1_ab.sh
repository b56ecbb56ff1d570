#!/bin/bash
# 1x1 conv GEMM autograd: its tests + model tests, then sampler/train bench A (BPK_GEMM1X1=0)
# vs B (default) twice on one box.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_1x1.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_1x1.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_1x1.log | head -20; exit $rc; }
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then E="BPK_GEMM1X1=0"; else E="BPK_GEMM1X1=1"; fi
    env $E timeout -k 10 400 python bench.py --steps 10 --train-steps 6 --no-pinn --no-dps --no-cpu-baseline > gpurun_out/ab1x1$v$i.log 2> gpurun_out/ab1x1$v$i.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab1x1$v$i.log'));print('$v', d['value'], d.get('train_steps_per_s'), d.get('cifar_train_steps_per_s'))"
  done
done
