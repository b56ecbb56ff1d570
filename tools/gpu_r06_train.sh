#!/bin/bash
# DSM / CIFAR train steps after the weight-gradient split changes: default (B=64 / 128) and the
# per-rank batches of the 8-GPU point (B=8 / 16)
set -o pipefail
O=gpurun_out/r06train; mkdir -p $O; export TMPDIR=/tmp
F="--no-pinn --no-dps --ns-steps 0 --ncddpmpp-steps 0 --no-cpu-baseline --steps 4 --warmup 2"
timeout -k 10 600 python3 bench.py $F > $O/b64.json 2> $O/b64.err || { tail -20 $O/b64.err; exit 1; }
timeout -k 10 600 python3 bench.py $F --per-rank-of 8 > $O/b8.json 2> $O/b8.err || { tail -20 $O/b8.err; exit 1; }
for f in b64 b8; do python3 -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', {k: d.get(k) for k in ('value','train_steps_per_s','cifar_train_steps_per_s')})"; done
