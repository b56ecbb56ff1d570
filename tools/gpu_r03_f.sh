#!/bin/bash
# r03: the multi-item 16-cin Winograd kernel (wino_f23_k16p_kernel): conv parity incl. the
# multi-item launches, the weighted PRE-conv mix with it (default) vs one item per workgroup
# (BPK_WINO_K16_IPW=1), and the per-workgroup timeline of both.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv3x3_winograd" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/k16p_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/k16p_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in 1 0; do
  BPK_WINO_K16_IPW=$v timeout -k 10 120 python tools/bench_wino_mix.py > gpurun_out/mix_ipw_$v.txt 2>&1 || { tail -5 gpurun_out/mix_ipw_$v.txt; exit 1; }
  echo "IPW=$v $(tail -1 gpurun_out/mix_ipw_$v.txt)"
done; done
cat gpurun_out/mix_ipw_0.txt
cat > /tmp/upf_ab.py <<'PY'
import sys, json, os
sys.path[:0] = ["b-pinn-kalman-filter_amd", "."]
import torch, bench
dev = torch.device("cuda:0")
r = bench.upfirdn_rooflines(dev, 64)
print(os.environ.get("BPK_UPFIRDN_R2", "4"), json.dumps([(x["kernel"][:28], x["frac"]) for x in r]))
PY
for r2 in 4 8 16 4 8 16; do BPK_UPFIRDN_R2=$r2 timeout -k 10 120 python /tmp/upf_ab.py || exit 1; done
