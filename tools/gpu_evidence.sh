#!/bin/bash
# Evidence for the judged numbers: the default bench command twice, the per-rank work of
# the 8-GPU point, rocprofv3 kernel summaries of the DSM train step (B = 64), DPS and the PINN
# graph step at B = 8.
set -o pipefail
O=${1:-gpurun_out/evidence}; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 900 python3 bench.py > $O/bench_$r.json 2> $O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  grep -o '"value": [0-9.]*' $O/bench_$r.json | head -1
done
timeout -k 10 900 python3 bench.py --per-rank-of 8 > $O/per_rank_of_8.json 2> $O/per_rank_of_8.err || { tail -20 $O/per_rank_of_8.err; exit 1; }
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/train -o train --output-format csv -- python3 tools/prof_train.py > $O/train.log 2>&1 || { tail -5 $O/train.log; exit 1; }
rm -f $O/train/train_kernel_trace.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/dps -o dps --output-format csv -- python3 tools/prof_dps.py 2 > $O/dps.log 2>&1 || { tail -5 $O/dps.log; exit 1; }
rm -f $O/dps/dps_kernel_trace.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p8 -o pinn --output-format csv -- python3 tools/prof_pinn.py graph 8 5 > $O/p8.log 2>&1 || { tail -5 $O/p8.log; exit 1; }
python3 tools/trace_steps.py $O/p8/pinn_kernel_trace.csv 5 45 > $O/p8_per_step.txt
rm -f $O/p8/pinn_kernel_trace.csv
head -2 $O/p8_per_step.txt
echo done
