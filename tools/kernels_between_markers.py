"""Per-kernel time between the two marker dispatches (fused_bias_act_kernel) that
tools/prof_steps.py puts around one counted bench step, from a rocprofv3 kernel trace CSV.
usage: kernels_between_markers.py kernel_trace.csv [top]"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
idx = [i for i, r in enumerate(rows) if "fused_bias_act" in r["Kernel_Name"]]
assert len(idx) >= 2, idx
sel = rows[idx[-2] + 1:idx[-1]]
span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e6
tot = defaultdict(float)
cnt = defaultdict(int)
for r in sel:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tot[r["Kernel_Name"]] += d
    cnt[r["Kernel_Name"]] += 1
busy = sum(tot.values())
print(f"{len(sel)} launches, span {span:.2f} ms, kernel-busy {busy:.2f} ms ({100 * busy / span:.1f} %)")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:top]:
    print(f"{100 * v / busy:6.2f}% {cnt[k]:6d} {1e3 * v / cnt[k]:9.1f} us  {k[:120]}")
