#!/bin/bash
# r03 session 2: L2 prefetch of the next block's first patches in the 16-cin Winograd kernel
# (BPK_WINO_PF=1) -- conv parity tests with it on, then the PRE-conv mix A/B, interleaved x3
mkdir -p gpurun_out; export TMPDIR=/tmp
BPK_WINO_PF=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -q -k "conv or wino or up2" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s10_test.log 2>&1; rc=$?
tail -2 gpurun_out/s10_test.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/s10_test.log | head; exit $rc; }
for r in 1 2 3; do
  for pf in 0 1; do
    BPK_WINO_PF=$pf timeout -k 10 300 python tools/bench_wino_mix.py > gpurun_out/s10_mix_${pf}_$r.log 2>&1 || { tail gpurun_out/s10_mix_${pf}_$r.log; exit 1; }
    echo "PF=$pf $(tail -1 gpurun_out/s10_mix_${pf}_$r.log)"
  done
done
grep -h "128->128@128\|256->256@64" gpurun_out/s10_mix_*_1.log
