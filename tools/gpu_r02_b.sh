#!/bin/bash
# upfirdn2d tail path + multi-rank tests, then the four upfirdn2d rooflines.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_dist.py -q -k "upfirdn or dist or shard or nan or simulator" --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_b.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "
import sys, json, torch; sys.argv=['bench']
import bench
for r in bench.upfirdn_rooflines(torch.device('cuda:0'), 64): print(json.dumps(r))
" || exit 1
