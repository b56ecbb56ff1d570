#!/bin/bash
# Round 5: is the PINN graph corruption a kernel-argument ring wrapping?  Fixed-parameter
# replays (tools/audit_pinn_graph.py iso) with eager launches of small / large kernel-argument
# blocks between them, then the failing case under three HIP runtime settings, then the PC
# sampler's step graph with eager reductions between steps.  Last: a PMC pass over the DPS step
# with a larger kernel-argument pool (its SIGSEGV was inside a launch, at a pool-sized boundary).
mkdir -p gpurun_out/r05b; export TMPDIR=/tmp
O=gpurun_out/r05b
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "pair_form or split_k or winograd" > $O/pytest_pair.log 2>&1 || { tail -30 $O/pytest_pair.log; exit 1; }
tail -2 $O/pytest_pair.log
run() {  # name, env..., -- args
  local name=$1; shift
  env "$@" timeout -k 10 240 python -u tools/audit_pinn_graph.py $ARGS > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }
  echo "$name: $(grep RESULT $O/$name.log)"
}
ARGS="iso fillflood 64" run fillflood
ARGS="iso ncflood 64" run ncflood
ARGS="iso redlarge_item 64" run pcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
ARGS="iso redlarge_item 64" run devka HIP_FORCE_DEV_KERNARG=1
ARGS="iso redlarge_item 64" run pool64 HSA_KERNARG_POOL_SIZE=67108864
ARGS="iso none 64" run none_pcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
ARGS="pc redlarge_item" run pc_red
if [ -n "$PMC" ]; then
  HSA_KERNARG_POOL_SIZE=67108864 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/dps_fetch -o pmc --output-format csv -- python3 tools/prof_steps.py dps > $O/dps_fetch.log 2>&1 || { tail -3 $O/dps_fetch.log; exit 1; }
  echo "dps fetch pass ok"
fi
