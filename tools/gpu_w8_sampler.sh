#!/bin/bash
# PC-sampler evals/s with the 8-wave Winograd form for PRE convs only (BPK_WINO_W8=1, default)
# vs every conv without a residual tail (=3), interleaved; conv tests under =3 first.
mkdir -p gpurun_out; export TMPDIR=/tmp
BPK_WINO_W8=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -k "conv3x3 or wino" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/w8s_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/w8s_pytest.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-train --no-pinn --no-dps --ns-steps 0 --ncddpmpp-steps 0 --steps 10 --warmup 2"
for r in 1 2; do for v in 1 3; do
  BPK_WINO_W8=$v timeout -k 10 300 python bench.py $B > gpurun_out/w8s_$v.log 2> gpurun_out/w8s_$v.err || { tail -5 gpurun_out/w8s_$v.err; exit 1; }
  echo "W8=$v $(grep -o '"value": [0-9.]*' gpurun_out/w8s_$v.log) $(grep -o '"frac": [0-9.]*' gpurun_out/w8s_$v.log | head -1)"
done; done
