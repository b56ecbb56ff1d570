#!/bin/bash
# persistent Winograd (BPK_WINO_PERSIST=1) correctness + sweep vs the default pipe kernel
mkdir -p gpurun_out; export TMPDIR=/tmp
BPK_WINO_PERSIST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "conv3x3_winograd" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_persist.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_persist.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_persist.log | head; exit $rc; }
BPK_WINO_PERSIST=1 timeout -k 10 300 python tools/bench_conv_sweep.py > gpurun_out/sweep1.log 2>&1 || { cat gpurun_out/sweep1.log; exit 1; }
echo "== persist"; grep cin gpurun_out/sweep1.log
timeout -k 10 300 python tools/bench_conv_sweep.py > gpurun_out/sweep0.log 2>&1 || exit 1
echo "== pipe"; grep cin gpurun_out/sweep0.log
for i in 1 2; do
  BPK_WINO_PERSIST=1 timeout -k 10 300 python bench.py --steps 20 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/abP$i.log 2> gpurun_out/abP$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abP$i.log'));print('persist', d['value'])"
  timeout -k 10 300 python bench.py --steps 20 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/abQ$i.log 2> gpurun_out/abQ$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abQ$i.log'));print('pipe', d['value'])"
done
