#!/bin/bash
# Round 6 (session 2): dense gradient pieces of the up-path skip concatenation -- parity tests,
# DSM / CIFAR train and DPS A/B (BPK_CAT_DENSE=0 / 1, interleaved x2).
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_dps.py -x -q --timeout 300 --timeout-method thread -k "cat_channels or gn_fanout or gn_silu_conv or cifar or train or dps or forward_pair" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ARGS="--steps 1 --warmup 1 --no-pinn --ns-steps 0 --ncddpmpp-steps 0 --no-cpu-baseline --no-roofline --train-steps 8 --cifar-steps 6 --dps-steps 3"
for r in 1 2; do
  for f in 0 1; do
    BPK_CAT_DENSE=$f timeout -k 10 600 python3 bench.py $ARGS > $O/t_f${f}_$r.json 2> $O/t_f${f}_$r.err || { tail -20 $O/t_f${f}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/t_f${f}_$r.json').read().strip().splitlines()[-1]); print('cat_dense $f run $r', 'dsm', d['train_steps_per_s'], 'cifar', d['cifar_train_steps_per_s'], 'dps', d['dps_nfe_per_s'], 'loss', d['train_loss'])"
  done
done
