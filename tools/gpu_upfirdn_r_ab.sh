#!/bin/bash
# upfirdn2d down2 two-column path: strip height 4 (default) vs 8 (BPK_UPFIRDN_R2=8), upfirdn
# tests under R=8, then the bench's upfirdn roofline line A/B twice.
mkdir -p gpurun_out; export TMPDIR=/tmp
BPK_UPFIRDN_R2=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k upfirdn -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_r.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_r.log | head; exit $rc; }
for i in 1 2; do for r in 4 8; do
  BPK_UPFIRDN_R2=$r timeout -k 10 300 python bench.py --steps 10 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/ur$r$i.log 2> gpurun_out/ur$r$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ur$r$i.log'));print('R=$r', d['value'], d['roofline_upfirdn2d']['ms_per_launch'], d['roofline_upfirdn2d']['frac'])"
done; done
