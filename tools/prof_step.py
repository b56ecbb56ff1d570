"""Per-PC-step kernel breakdown from a rocprofv3 kernel trace: kernels between the last
(n+1) `k_step_inc` dispatches (the timed graph replays), grouped by kernel name."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
inc = [i for i, r in enumerate(rows) if "k_step_inc" in r["Kernel_Name"]]
lo, hi = inc[-(n + 1)], inc[-1]
sel = rows[lo + 1:hi + 1]
agg = defaultdict(lambda: [0, 0])
for r in sel:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[r["Kernel_Name"]][0] += d
    agg[r["Kernel_Name"]][1] += 1
busy = sum(v[0] for v in agg.values())
wall = int(sel[-1]["End_Timestamp"]) - int(rows[lo]["End_Timestamp"])
print(f"{n} PC steps: wall {wall/1e6:.2f} ms  kernel-busy {busy/1e6:.2f} ms  ({busy/wall*100:.1f}%)"
      f"  per step {wall/n/1e6:.2f} ms, {len(sel)/n:.0f} launches/step")
for name, (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{d/busy*100:6.2f}%  {c/n:6.1f}/step  {d/c/1e3:9.1f} us  {name[:100]}")
