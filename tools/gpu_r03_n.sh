#!/bin/bash
# r03: static Winograd filters in the sampler graph + aligned FIR stores: tests, A/B, bench
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_dist.py -k "pc_engine or graph or sampler or pc_" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/n_tests.log 2>&1; rc=$?; echo "model tests: $(tail -1 gpurun_out/n_tests.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/n_tests.log | head; exit $rc; }
TESTENV=BPK_UPFIRDN_FIR_ALIGN=1 bash tools/gpu_upfirdn_roll.sh BPK_UPFIRDN_FIR_ALIGN=1 || exit 1
timeout -k 10 600 python bench.py --steps 10 --no-train --no-pinn --no-dps --ns-steps 0 --no-cpu-baseline > gpurun_out/n_bench.log 2> gpurun_out/n_bench.err || { tail -5 gpurun_out/n_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/n_bench.log'));print('bench', d['value'], d['roofline']['frac'], d.get('ncddpmpp_evals_per_s'), [(r['kernel'][:22], r['frac']) for r in d.get('roofline_upfirdn2d', [])])"
