#!/bin/bash
# Round 6 rocprofv3 kernel summaries on the final tree: PC sampler at B=64 / the per-rank B=8,
# DSM train (B=64, B=8), CIFAR train, DPS and the PINN graph step (B=64, B=8).
set -o pipefail
O=gpurun_out/r06prof; mkdir -p $O; export TMPDIR=/tmp; export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
prof() {  # name limit keep_trace -- command
  local name=$1 lim=$2 keep=$3; shift 4
  timeout -k 10 $lim rocprofv3 --kernel-trace --stats -d $O/$name -o $name --output-format csv -- "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name ok"
  [ "$keep" = 1 ] || rm -f $O/$name/${name}_kernel_trace.csv
}
SAMPLER="--no-cpu-baseline --no-train --no-pinn --no-dps --cifar-steps 0 --ns-steps 0 --ncddpmpp-steps 0 --no-roofline"
prof b64 400 0 -- python3 bench.py --steps 4 --warmup 2 $SAMPLER
prof b8 400 0 -- python3 bench.py --steps 4 --warmup 2 --global-batch 8 $SAMPLER
prof train 400 0 -- python3 tools/prof_train.py
prof train_b8 300 0 -- python3 tools/prof_train.py 8
prof cifar 400 0 -- python3 tools/prof_cifar.py
prof dps 400 0 -- python3 tools/prof_dps.py 2
prof pinn 300 1 -- python3 tools/prof_pinn.py graph 1 5
python3 tools/trace_steps.py $O/pinn/pinn_kernel_trace.csv 5 45 > $O/pinn_per_step.txt
rm -f $O/pinn/pinn_kernel_trace.csv
prof pinn_b8 300 1 -- python3 tools/prof_pinn.py graph 8 5
python3 tools/trace_steps.py $O/pinn_b8/pinn_b8_kernel_trace.csv 5 45 > $O/pinn_b8_per_step.txt
rm -f $O/pinn_b8/pinn_b8_kernel_trace.csv
