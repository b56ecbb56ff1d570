#!/bin/bash
# r03 round-end check, part 1: the whole GPU test suite and smoke()
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/final_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/final_pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/final_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/final_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/final_smoke.log; exit $rc
