#!/bin/bash
# Round-end evidence: default N=1 bench (as the driver runs it), smoke(), sampler kernel trace.
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_bench.sh noprof || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" || exit 1
bash tools/gpu_prof_sampler.sh > /dev/null || exit 1
echo SAMP_PROF_OK
bash tools/gpu_prof_train2.sh || exit 1
