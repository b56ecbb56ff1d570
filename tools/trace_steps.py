"""Per-step kernel count and busy time of the timed graph replays in a rocprofv3 kernel trace
of tools/prof_pinn.py: the periods between the step's FilterBatch launches (else: segments
separated by > 2 ms of idle, the longest holding the replays): python tools/trace_steps.py
TRACE.csv REPLAYS [TOP]"""
import collections
import csv
import re
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    if "at::native" in n:
        m = re.search(r"at::native::(?:\(anonymous namespace\)::)?(\w+)<[^,]*,\s*at::native::([\w:]+)", n)
        return "aten:" + (m.group(2) if m else n[:60])
    return n.split("(")[0][:70]


rows = list(csv.DictReader(open(sys.argv[1])))
nrep = int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
segs, cur, last = [], [ev[0]], ev[0][1]
for e in ev[1:]:
    if e[0] - last > 2_000_000:
        segs.append(cur)
        cur = []
    cur.append(e)
    last = max(last, e[1])
segs.append(cur)
s = max(segs, key=len)
# the graph step starts with the one FilterBatch launch (every Winograd filter of the step):
# when present, a step is the period between two of them (the replay plus the eager optimizer
# / EMA launches after it); the last nrep periods are the timed replays
marks = [i for i, e in enumerate(ev) if "wino_filter_batch_kernel" in e[2]]
if len(marks) > nrep:
    s = ev[marks[-nrep - 1]:marks[-1]]
t, c = collections.Counter(), collections.Counter()
for e in s:
    k = short(e[2])
    t[k] += e[1] - e[0]
    c[k] += 1
tot = sum(t.values())
print(f"per step: {tot / nrep / 1e6:.1f} ms busy, {len(s) / nrep:.0f} kernels, "
      f"{(s[-1][1] - s[0][0]) / nrep / 1e6:.1f} ms span (under the profiler)")
at = sum(v for k, v in t.items() if k.startswith("aten"))
ac = sum(c[k] for k in t if k.startswith("aten"))
print(f"aten: {at / nrep / 1e6:.2f} ms, {ac / nrep:.0f} launches per step")
for k, v in t.most_common(top):
    print(f"{v / nrep / 1e6:7.2f} ms {c[k] / nrep:7.0f} {v / c[k] / 1e3:7.1f}us  {k}")
