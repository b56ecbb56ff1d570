#!/bin/bash
# Round 6: PINN step with the residual's derivative passes batched over input copies
# (BPK_PINN_COPIES) and the two frames' pyramids as one batch (BPK_PAIR_FRAMES): parity tests,
# then graph-step timing at the per-rank B=8 and at B=64.
set -o pipefail
O=gpurun_out/r06copies; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_pinn.py -k graph tests/test_gpu_graph.py > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
run() { # name per-rank-of env...
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 300 python3 tools/prof_pinn.py graph $n 20 > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  echo "$name: $(grep -o "'pinn_train_steps_per_s': [0-9.]*" $O/$name.log) $(grep -o "'pinn_losses': [^]]*" $O/$name.log)"
}
run b8_c1 8 BPK_PINN_COPIES=1
run b8_c2 8 BPK_PINN_COPIES=2
run b8_c4 8 BPK_PINN_COPIES=4
run b8_c4_nopair 8 BPK_PINN_COPIES=4 BPK_PAIR_FRAMES=0
run b64_c1 1 BPK_PINN_COPIES=1
run b64_c1_nopair 1 BPK_PINN_COPIES=1 BPK_PAIR_FRAMES=0
run b64_c2 1 BPK_PINN_COPIES=2
run b64_c4 1 BPK_PINN_COPIES=4
# ns_step with the XCD-ordered tiles: bit-exact tests, time, HBM traffic (separate PMC passes)
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "ns_" > $O/ns_tests.log 2>&1 || { tail -30 $O/ns_tests.log; exit 1; }
tail -1 $O/ns_tests.log
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train --no-pinn --no-dps --cifar-steps 0 --ncddpmpp-steps 0 --no-roofline --ns-steps 50 > $O/ns_bench.log 2>&1 || { tail -20 $O/ns_bench.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$O/ns_bench.log').read().strip().splitlines()[-1]); print({k: d[k] for k in ('ns_gsites_per_s','ns_ms_per_step')})"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $O/ns_$ctr -o pmc --output-format csv -- python3 tools/prof_r02.py ns > $O/ns_$ctr.log 2>&1 || { tail -5 $O/ns_$ctr.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r06copies/ns_*/**/*counter_collection*.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(k, c, len(v), sum(v) / len(v))
PY
