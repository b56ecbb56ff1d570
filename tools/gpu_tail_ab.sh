#!/bin/bash
# Peeled tail chunks in the Winograd PRE conv (BPK_WINO_TAIL=1, default) vs none (=0): conv
# parity tests, then the census mix (tools/bench_wino_mix.py) interleaved.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -k "conv3x3 or wino" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tail_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/tail_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in 0 1; do
  BPK_WINO_TAIL=$v timeout -k 10 200 python tools/bench_wino_mix.py > gpurun_out/tail_mix_$v.txt 2>&1 || { tail -5 gpurun_out/tail_mix_$v.txt; exit 1; }
  echo "TAIL=$v $(tail -1 gpurun_out/tail_mix_$v.txt)"
done; done
