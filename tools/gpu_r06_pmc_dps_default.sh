#!/bin/bash
# Does the DPS step's PMC pass still die at the default kernel-argument pool size once the graph
# packet-capture setting is in effect for the profiler-started runtime?  
set -o pipefail
O=gpurun_out/r06pmcdps; mkdir -p $O; export TMPDIR=/tmp
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
unset HSA_KERNARG_POOL_SIZE
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/dps_fetch -o pmc --output-format csv -- python3 tools/prof_steps.py dps > $O/dps_fetch.log 2>&1
rc=$?
echo "dps FETCH_SIZE pass at the default pool, packet capture off: rc=$rc"
grep -c "fused_bias_act_kernel<double>" $O/dps_fetch/pmc_counter_collection.csv 2>/dev/null || true
grep -m3 -i "SIGSEGV\|Aborted" $O/dps_fetch.log || true
