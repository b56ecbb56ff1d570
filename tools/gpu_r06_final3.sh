#!/bin/bash
# Round 6, second session, final tree: the driver's default bench command twice, the per-rank
# work of the 8-GPU point, rocprofv3 kernel traces of the PINN graph step at B = 64 and B = 8.
set -o pipefail
O=gpurun_out/r06final3; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 900 python3 bench.py > $O/bench_$r.json 2> $O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  grep -o '"value": [0-9.]*' $O/bench_$r.json | head -1
done
timeout -k 10 900 python3 bench.py --per-rank-of 8 > $O/per_rank_of_8.json 2> $O/per_rank_of_8.err || { tail -20 $O/per_rank_of_8.err; exit 1; }
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
for n in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$n -o pinn --output-format csv -- python3 tools/prof_pinn.py graph $n 5 > $O/p$n.log 2>&1 || { tail -5 $O/p$n.log; exit 1; }
  python3 tools/trace_steps.py $O/p$n/pinn_kernel_trace.csv 5 45 > $O/p${n}_per_step.txt
  head -2 $O/p${n}_per_step.txt
  rm -f $O/p$n/pinn_kernel_trace.csv
done
echo done
