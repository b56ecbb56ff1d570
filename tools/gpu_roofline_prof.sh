#!/bin/bash
# The roofline kernel two ways on one box: bench.py's in-run HIP-event timing of the
# 128->128 @128^2 B=64 Winograd conv, and the rocprofv3 kernel-trace summary of the same
# kernel / shape launched 20 times (tools/prof_conv.py).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 5 --no-train --no-pinn --no-dps --no-cpu-baseline > gpurun_out/roof_bench.json 2> gpurun_out/roof_bench.err || { tail -5 gpurun_out/roof_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/roof_bench.json'));print('bench roofline ms/launch', d['roofline']['ms_per_launch'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_roof -o roof --output-format csv -- python tools/prof_conv.py > gpurun_out/prof_roof.log 2>&1 || { tail -5 gpurun_out/prof_roof.log; exit 1; }
python - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof_roof/roof_kernel_stats.csv")):
    if "wino_f23" in r["Name"]:
        print("rocprof", r["Name"][:60], r["Calls"], "avg ms", float(r["AverageNs"]) / 1e6)
PY
