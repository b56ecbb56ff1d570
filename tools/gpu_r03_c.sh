#!/bin/bash
# r03: the 16-cin chunk 8-wave Winograd kernel (BPK_WINO_K16): conv parity with it forced on
# every supported launch, then the weighted PRE-conv mix A/B vs the 8-cin form.
mkdir -p gpurun_out; export TMPDIR=/tmp
BPK_WINO_K16=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv3x3_winograd" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/k16_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/k16_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in 0 1; do
  BPK_WINO_K16=$v timeout -k 10 120 python tools/bench_wino_mix.py > gpurun_out/mix_k16_$v.txt 2>&1 || { tail -5 gpurun_out/mix_k16_$v.txt; exit 1; }
  echo "K16=$v $(tail -1 gpurun_out/mix_k16_$v.txt)"
done; done
cat gpurun_out/mix_k16_1.txt
