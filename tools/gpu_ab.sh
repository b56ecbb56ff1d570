#!/bin/bash
# Same-box A/B of one environment switch over bench.py phases, interleaved.
#   tools/gpu_ab.sh OUT VAR "VALUES" REPEATS [bench.py args...]
# e.g. tools/gpu_ab.sh gpurun_out/ab BPK_GN_FANOUT "0 1" 2 --no-pinn --no-dps --ns-steps 0 \
#        --ncddpmpp-steps 0 --no-cpu-baseline --no-roofline --train-steps 8 --cifar-steps 6
# The round's switches: BPK_DEFER_WGRAD, BPK_GN_FANOUT, BPK_IN_FANOUT, BPK_PINN_COPIES,
# BPK_GN_CONV_AD_TRAIN.  Each run's JSON line goes to OUT/<VAR>_<value>_<repeat>.json and
# every "*_per_s" rate of it is printed.
set -o pipefail
O=$1; VAR=$2; VALS=$3; REP=$4; shift 4
mkdir -p "$O"; export TMPDIR=/tmp
for r in $(seq 1 "$REP"); do
  for v in $VALS; do
    f="$O/${VAR}_${v}_$r"
    env "$VAR=$v" timeout -k 10 900 python3 bench.py "$@" > "$f.json" 2> "$f.err" || { tail -20 "$f.err"; exit 1; }
    python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'run', sys.argv[3], {k: v for k, v in d.items() if k.endswith('_per_s') or k == 'value'})" \
      "$f.json" "$VAR=$v" "$r"
  done
done
