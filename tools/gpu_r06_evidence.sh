#!/bin/bash
# Round 6 evidence: rocprofv3 kernel summaries of the PINN graph step at the per-rank B=8 and at
# B=64, the DSM train step at the per-rank B=8, and the bench's per-rank-of-8 line.
set -o pipefail
O=gpurun_out/r06ev; mkdir -p $O; export TMPDIR=/tmp
prof() {  # name limit -- command
  local name=$1 lim=$2; shift 3
  timeout -k 10 $lim rocprofv3 --kernel-trace --stats -d $O/$name -o $name --output-format csv -- "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name ok: $(grep -v '^[WE]2026' $O/$name.log | tail -1 | cut -c1-200)"
}
prof pinn_b8 300 -- python3 tools/prof_pinn.py graph 8 5
python3 tools/trace_steps.py $O/pinn_b8/pinn_b8_kernel_trace.csv 5 45 > $O/pinn_b8_per_step.txt 2>&1 || true
prof pinn_b64 300 -- python3 tools/prof_pinn.py graph 1 5
python3 tools/trace_steps.py $O/pinn_b64/pinn_b64_kernel_trace.csv 5 45 > $O/pinn_b64_per_step.txt 2>&1 || true
prof train_b8 300 -- python3 tools/prof_train.py 8
rm -f $O/train_b8/train_b8_kernel_trace.csv
timeout -k 10 900 python3 bench.py --per-rank-of 8 --no-cpu-baseline > $O/per_rank_of_8.json 2> $O/per_rank_of_8.err || { tail -20 $O/per_rank_of_8.err; exit 1; }
tail -c 600 $O/per_rank_of_8.json
