#!/bin/bash
# Round 4: the whole GPU test suite, then the default N=1 bench line (as the driver runs it);
# each step under its own limit, stop at the first failure.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
[ "$1" = "tests" ] && exit 0
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.log
