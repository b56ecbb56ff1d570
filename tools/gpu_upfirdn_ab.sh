#!/bin/bash
# upfirdn2d down2 two-columns-per-lane path: GPU tests, then sampler + upfirdn roofline A/B
# (A: BPK_UPFIRDN_NOC1=1, one column per lane; B: default).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_up.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_up.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_up.log | head; exit $rc; }
for i in 1 2; do
  BPK_UPFIRDN_NOC1=1 timeout -k 10 300 python bench.py --steps 20 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/upA$i.log 2> gpurun_out/upA$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/upA$i.log'));print('A', d['value'], d['roofline_upfirdn2d']['ms_per_launch'], d['roofline_upfirdn2d']['frac'])"
  timeout -k 10 300 python bench.py --steps 20 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/upB$i.log 2> gpurun_out/upB$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/upB$i.log'));print('B', d['value'], d['roofline_upfirdn2d']['ms_per_launch'], d['roofline_upfirdn2d']['frac'])"
done
