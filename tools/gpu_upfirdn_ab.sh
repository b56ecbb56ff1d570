#!/bin/bash
# upfirdn2d A/B over env variants (tools/bench_upfirdn.py); "$@" = variants as VAR=VALUE,...
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in base "$@"; do
  envs=$(echo "$v" | tr ',' ' '); [ "$v" = base ] && envs=""
  env $envs TAG="$v" timeout -k 10 120 python tools/bench_upfirdn.py 2>/dev/null || { echo "variant $v failed"; exit 1; }
done
