#!/bin/bash
# r03 session 2 round-end evidence: the whole GPU suite + smoke, the default N=1 bench line,
# then the sampler-only rocprofv3 kernel trace (tools/gpu_bench.sh)
bash tools/gpu_r03_final_tests.sh || exit 1
bash tools/gpu_bench.sh prof sampler_only_s2 || exit 1
