#!/bin/bash
# 8-wave Winograd workgroup A/B on the NCSN++ PRE-conv mix (tools/bench_wino_mix.py), interleaved.
mkdir -p gpurun_out; export TMPDIR=/tmp
BPK_WINO_W8=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -k "conv3x3 or wino" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/w8_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/w8_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in 0 1; do
  BPK_WINO_W8=$v timeout -k 10 200 python tools/bench_wino_mix.py > gpurun_out/w8_mix_$v.txt 2>&1 || { tail -5 gpurun_out/w8_mix_$v.txt; exit 1; }
  echo "W8=$v $(tail -1 gpurun_out/w8_mix_$v.txt)"
done; done
