#!/bin/bash
# Round 6 (session 2): fixed-order gamma / beta sums in the resident GroupNorm backward --
# tests (determinism, fp64 reference, the fan-out bit-identity), DSM / CIFAR / DPS timing.
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "group_norm or gn_ or cifar or train or dps or biggan or ddpm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ARGS="--steps 1 --warmup 1 --no-pinn --ns-steps 0 --ncddpmpp-steps 0 --no-cpu-baseline --no-roofline --train-steps 8 --cifar-steps 6 --dps-steps 3"
for r in 1 2; do
  timeout -k 10 600 python3 bench.py $ARGS > $O/t_$r.json 2> $O/t_$r.err || { tail -20 $O/t_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/t_$r.json').read().strip().splitlines()[-1]); print('run $r', 'dsm', d['train_steps_per_s'], 'cifar', d['cifar_train_steps_per_s'], 'dps', d['dps_nfe_per_s'], 'loss', d['train_loss'])"
done
