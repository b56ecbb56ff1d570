#!/bin/bash
# upfirdn2d up2 four-column path: upfirdn tests, then timing A (BPK_UPFIRDN_UP2=1) vs B, and
# the sampler bench A/B.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_up2.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_up2.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_up2.log | head; exit $rc; }
echo "== A"; BPK_UPFIRDN_UP2=1 timeout -k 10 120 python tools/bench_up2.py || exit 1
echo "== B"; timeout -k 10 120 python tools/bench_up2.py || exit 1
for i in 1 2; do
  BPK_UPFIRDN_UP2=1 timeout -k 10 300 python bench.py --steps 20 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/u2A$i.log 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/u2A$i.log'));print('A', d['value'])"
  timeout -k 10 300 python bench.py --steps 20 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/u2B$i.log 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/u2B$i.log'));print('B', d['value'])"
done
