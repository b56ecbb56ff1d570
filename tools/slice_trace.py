"""Steady-state kernel breakdown from a rocprofv3 kernel trace: drop everything up to the
end of the warm-up, located as occurrence (per_step * warmup) of a marker kernel that runs a
fixed number of times per step.
usage: slice_trace.py trace.csv marker per_step warmup steps [top]  (per_step 0: inferred)"""
import csv
import sys
from collections import defaultdict

path, marker = sys.argv[1], sys.argv[2]
per_step, warmup, steps = int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
top = int(sys.argv[6]) if len(sys.argv) > 6 else 25
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
if per_step == 0:  # infer: the marker's total count over warmup + steps
    per_step = len(idx) // (warmup + steps)
# counted from the end: the last `steps` steps hold per_step * steps marker launches (extra
# marker launches before the warm-up, e.g. an initialisation, do not shift the slice)
assert len(idx) >= per_step * (warmup + steps), (len(idx), per_step * (warmup + steps))
lo = idx[len(idx) - per_step * steps - 1] + 1
sel = rows[lo:]
agg = defaultdict(lambda: [0, 0])
for r in sel:
    agg[r["Kernel_Name"]][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[r["Kernel_Name"]][1] += 1
busy = sum(v[0] for v in agg.values())
wall = int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])
print(f"{steps} steps: wall {wall / 1e6:.1f} ms, kernel-busy {busy / 1e6:.1f} ms "
      f"({busy / wall * 100:.1f} %), {len(sel) / steps:.0f} launches/step")
for name, (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
    print(f"{d / busy * 100:6.2f}%  {c / steps:7.1f}/step  {d / c / 1e3:9.1f} us  {name[:100]}")
