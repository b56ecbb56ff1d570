#!/bin/bash
# Round-end check: every -m gpu test, smoke(), the default bench line, and the rocprofv3
# kernel-trace stats of the sampler phase (bench.py --no-train ... under the profiler).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" || exit 1
bash tools/gpu_bench.sh || exit 1
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof/bench_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:8]:
    print(f'{float(r["TotalDurationNs"]) / tot * 100:6.2f}%  {r["Calls"]:>7}  {float(r["AverageNs"]) / 1e3:9.1f} us  {r["Name"][:90]}')
PY
