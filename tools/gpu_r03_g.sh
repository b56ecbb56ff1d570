#!/bin/bash
# r03: the default bench line (K16 Winograd everywhere it fits, fused attention), the PINN step
# as a hipGraph replay (20 replays, losses in the line), and the rocprofv3 kernel trace of the
# DSM train-step phase alone.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/bench_g.log 2> gpurun_out/bench_g.err || { tail -20 gpurun_out/bench_g.err; exit 1; }
cat gpurun_out/bench_g.log
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-train --no-dps --ns-steps 0 --ncddpmpp-steps 0 --no-roofline --no-cpu-baseline --pinn-graph --pinn-steps 20 > gpurun_out/bench_pinn_graph.log 2> gpurun_out/bench_pinn_graph.err || { tail -20 gpurun_out/bench_pinn_graph.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_pinn_graph.log').read().strip().splitlines()[-1]); print({k: d[k] for k in d if k.startswith('pinn')})"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_g -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 --no-roofline --no-cpu-baseline --no-pinn --no-dps --ns-steps 0 --ncddpmpp-steps 0 --cifar-steps 0 --train-steps 6 --train-warmup 2 > gpurun_out/prof_train_g.log 2>&1 || exit 1
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_train_g/bench_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:16]:
    print(f'{float(r["TotalDurationNs"]) / tot * 100:6.2f}%  {r["Calls"]:>7}  {float(r["AverageNs"]) / 1e3:9.1f} us  {r["Name"][:90]}')
PY
