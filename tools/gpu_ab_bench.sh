#!/bin/bash
# A/B of the sampler bench on one box: $1 = env assignment for variant B (variant A = defaults).
mkdir -p gpurun_out; export TMPDIR=/tmp
true
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/abA$i.log 2> gpurun_out/abA$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abA$i.log'));print('A', d['value'], d['roofline']['ms_per_launch'])"
  env $1 timeout -k 10 300 python bench.py --steps 20 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/abB$i.log 2> gpurun_out/abB$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abB$i.log'));print('B', d['value'], d['roofline']['ms_per_launch'])"
done
