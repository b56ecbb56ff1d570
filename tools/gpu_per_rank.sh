#!/bin/bash
# Per-rank work of the 2-, 4- and 8-GPU points on one GPU (bench.py --per-rank-of N) beside
# the 1-GPU line, interleaved REP times on one box, so each point of the driver's scaling run
# has a stated expectation.
set -o pipefail
O=${1:-gpurun_out/per_rank}; mkdir -p $O; export TMPDIR=/tmp
for r in $(seq 1 ${REP:-2}); do
for n in ${NS:-1 2 4 8}; do
  f=$O/per_rank_of_${n}_$r
  timeout -k 10 600 python3 bench.py --per-rank-of $n --no-cpu-baseline > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('per-rank-of', sys.argv[2], {k: v for k, v in d.items() if k.endswith('_per_s') or k == 'value'})" $f.json $n
done
done
