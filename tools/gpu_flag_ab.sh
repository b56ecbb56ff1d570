#!/bin/bash
# $1 = env flag (default on): GPU tests, then sampler bench A ($1=0) vs B ($1=1) twice on one box.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_flag.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_flag.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_flag.log | head -20; exit $rc; }
for i in 1 2; do
  for v in 0 1; do
    env $1=$v timeout -k 10 300 python bench.py --steps 20 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/abf$v$i.log 2> gpurun_out/abf$v$i.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/abf$v$i.log'));print('$1=$v', d['value'], d['ms_per_step'])"
  done
done
