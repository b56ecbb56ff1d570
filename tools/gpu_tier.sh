#!/bin/bash
# The driver's round-end GPU tier, rehearsed: pytest -m gpu, then smoke().
set -o pipefail
O=${1:-gpurun_out/gputier}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 600 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
