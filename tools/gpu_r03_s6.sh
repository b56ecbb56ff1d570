#!/bin/bash
# r03 session 2: the whole GPU suite (optionally filtered: $1 = pytest -k expression) and
# smoke(), then the 1x1 GEMM per-shape rates
mkdir -p gpurun_out; export TMPDIR=/tmp
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s6_pytest.log 2>&1; rc=$?
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s6_pytest.log 2>&1; rc=$?
fi
tail -3 gpurun_out/s6_pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/s6_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/s6_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/s6_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/s6_gemm.log 2>&1 || { tail gpurun_out/s6_gemm.log; exit 1; }
cat gpurun_out/s6_gemm.log
