#!/bin/bash
# Round 5 rocprofv3 kernel summaries: PC sampler at B=64 and at the per-rank B=8, DSM train,
# CIFAR train, DPS and PINN (graph replays).  Output: gpurun_out/r05prof/<name>/.
mkdir -p gpurun_out/r05prof; export TMPDIR=/tmp
O=gpurun_out/r05prof
prof() {  # name limit -- command
  local name=$1 lim=$2; shift 3
  timeout -k 10 $lim rocprofv3 --kernel-trace --stats -d $O/$name -o $name --output-format csv -- "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  echo "$name ok: $(grep -v '^[WE]2026' $O/$name.log | tail -1 | cut -c1-300)"
  [ "$name" = pinn ] || rm -f $O/$name/${name}_kernel_trace.csv
}
SAMPLER="--no-cpu-baseline --no-train --no-pinn --no-dps --cifar-steps 0 --ns-steps 0 --ncddpmpp-steps 0 --no-roofline"
prof b64 400 -- python3 bench.py --steps 4 --warmup 2 $SAMPLER
prof b8 400 -- python3 bench.py --steps 4 --warmup 2 --global-batch 8 $SAMPLER
prof train 400 -- python3 tools/prof_train.py
prof cifar 400 -- python3 tools/prof_cifar.py
prof dps 400 -- python3 tools/prof_dps.py 2
prof pinn 300 -- python3 tools/prof_pinn.py
