#!/bin/bash
# TembBank under autograd (training, DPS): parity tests, then A/B of the DSM / CIFAR / DPS phases
set -o pipefail
O=gpurun_out/r06tb; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_configs.py -k "cifar or dps" tests/test_gpu_models.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -20; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
F="--no-pinn --ns-steps 0 --ncddpmpp-steps 0 --no-cpu-baseline --steps 4 --warmup 2"
for v in 1 0; do
  for pr in "" "--per-rank-of 8"; do
    n=tb${v}_$( [ -z "$pr" ] && echo b64 || echo b8 )
    BPK_TEMB_BANK_AD=$v timeout -k 10 700 python3 bench.py $F $pr > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', {k: d.get(k) for k in ('value','train_steps_per_s','cifar_train_steps_per_s','dps_nfe_per_s')})"
  done
done
