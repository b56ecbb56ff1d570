#!/bin/bash
# r03 session 2: the fused nearest-upsample conv tests, the whole GPU suite + smoke, then the
# bench line (N=1).  Each GPU step has its own limit; stop at the first failure.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "up2 or upsample" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s2_up2.log 2>&1; rc=$?
tail -2 gpurun_out/s2_up2.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/s2_up2.log | head -20; exit $rc; }
[ "$1" = "full" ] && { bash tools/gpu_r03_final_tests.sh || exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/s2_bench.log 2> gpurun_out/s2_bench.err || { tail -20 gpurun_out/s2_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/s2_bench.log'));print('bench', d['value'], d['roofline']['frac'], d.get('ncddpmpp_evals_per_s'), d.get('dps_nfe_per_s'), d.get('train_steps_per_s'), [(r['kernel'][:22], r['frac']) for r in d.get('roofline_upfirdn2d', [])])"
