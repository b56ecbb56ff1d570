#!/bin/bash
# A/B of the sampler bench on one box: $1 = env assignment for variant B (variant A = defaults).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "conv3x3" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_conv.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_conv.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/abA$i.log 2> gpurun_out/abA$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abA$i.log'));print('A', d['value'], d['roofline']['ms_per_launch'])"
  env $1 timeout -k 10 300 python bench.py --steps 20 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/abB$i.log 2> gpurun_out/abB$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abB$i.log'));print('B', d['value'], d['roofline']['ms_per_launch'])"
done
