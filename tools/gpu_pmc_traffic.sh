#!/bin/bash
# HBM traffic of the two roofline kernels (tools/prof_traffic.py): FETCH_SIZE and WRITE_SIZE
# in separate rocprofv3 --pmc passes, averaged per kernel (KB per dispatch).
mkdir -p gpurun_out/pmct; export TMPDIR=/tmp
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/pmct/p$i -o pmc --output-format csv -- python tools/prof_traffic.py > gpurun_out/pmct/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmct/p$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmct/p*/**/*counter_collection*.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"][:50], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(f, k, c, len(v), sum(v) / len(v))
PY
