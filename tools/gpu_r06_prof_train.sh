#!/bin/bash
set -o pipefail
O=gpurun_out/r06pt; mkdir -p $O; export TMPDIR=/tmp; export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
prof() {  # name limit -- command
  local name=$1 lim=$2; shift 3
  timeout -k 10 $lim rocprofv3 --kernel-trace --stats -d $O/$name -o $name --output-format csv -- "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  rm -f $O/$name/${name}_kernel_trace.csv
  echo "$name ok"
}
prof train_b8 300 -- python3 tools/prof_train.py 8
prof train_b64 400 -- python3 tools/prof_train.py 64
prof cifar 400 -- python3 tools/prof_cifar.py
