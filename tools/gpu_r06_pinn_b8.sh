#!/bin/bash
# Round 6: PINN step at the per-rank B=8 (configs[3] sharded 8 ways) -- timing with the HIP
# runtime's graph packet capture off (the shipped setting) and on (timing only: replays with it
# on are not trusted, op/_hipenv.py), then a rocprofv3 kernel trace of the shipped setting.
set -o pipefail
O=gpurun_out/r06pinn; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/prof_pinn.py graph 8 20 > $O/b8_pc0.log 2>&1 || { tail -20 $O/b8_pc0.log; exit 1; }
tail -1 $O/b8_pc0.log
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 300 python3 tools/prof_pinn.py graph 8 20 > $O/b8_pc1.log 2>&1 || { tail -20 $O/b8_pc1.log; exit 1; }
tail -1 $O/b8_pc1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o pinn_b8 --output-format csv -- python3 tools/prof_pinn.py graph 8 5 > $O/prof_b8.log 2>&1 || { tail -20 $O/prof_b8.log; exit 1; }
tail -1 $O/prof_b8.log
