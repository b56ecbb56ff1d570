#!/bin/bash
# r03: every -m gpu test with the K16 Winograd default and the fused attention kernel, the
# default bench line, then the sampler-phase-only rocprofv3 kernel trace.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench.sh prof sampler_e || exit 1
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_sampler_e/bench_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"]) / tot * 100:6.2f}%  {r["Calls"]:>7}  {float(r["AverageNs"]) / 1e3:9.1f} us  {r["Name"][:90]}')
PY
