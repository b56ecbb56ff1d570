#!/bin/bash
# Round 6 (session 2): GroupNorm fan-out in the training-mode residual blocks -- parity tests,
# DSM / CIFAR train A/B (BPK_GN_FANOUT=0 / 1, interleaved x2).
set -o pipefail
O=gpurun_out/r06i; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "gn_fanout or gn_silu_conv or cifar or train or biggan or ddpm or dps" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ARGS="--steps 1 --warmup 1 --no-pinn --no-dps --ns-steps 0 --ncddpmpp-steps 0 --no-cpu-baseline --no-roofline --train-steps 8 --cifar-steps 6"
for r in 1 2; do
  for f in 0 1; do
    BPK_GN_FANOUT=$f timeout -k 10 600 python3 bench.py $ARGS > $O/t_f${f}_$r.json 2> $O/t_f${f}_$r.err || { tail -20 $O/t_f${f}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/t_f${f}_$r.json').read().strip().splitlines()[-1]); print('fanout $f run $r', 'dsm', d['train_steps_per_s'], 'cifar', d['cifar_train_steps_per_s'], 'loss', d['train_loss'])"
  done
done
for f in 0 1; do
  BPK_GN_FANOUT=$f timeout -k 10 600 python3 bench.py $ARGS --per-rank-of 8 > $O/p8_f${f}.json 2> $O/p8_f${f}.err || { tail -20 $O/p8_f${f}.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/p8_f${f}.json').read().strip().splitlines()[-1]); print('fanout $f per-rank-of-8', 'dsm', d['train_steps_per_s'], 'cifar', d['cifar_train_steps_per_s'])"
done
DARGS="--steps 1 --warmup 1 --no-train --cifar-steps 0 --no-pinn --ns-steps 0 --ncddpmpp-steps 0 --no-cpu-baseline --no-roofline --dps-steps 3"
for r in 1 2; do
  for f in 0 1; do
    BPK_GN_FANOUT=$f timeout -k 10 600 python3 bench.py $DARGS > $O/d_f${f}_$r.json 2> $O/d_f${f}_$r.err || { tail -20 $O/d_f${f}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/d_f${f}_$r.json').read().strip().splitlines()[-1]); print('fanout $f run $r', 'dps', d['dps_nfe_per_s'])"
  done
done
