"""Top kernels of a rocprofv3 --stats kernel summary: python tools/kstats.py FILE.csv [TOP]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{sys.argv[1]}: {tot / 1e6:.1f} ms kernel time, {sum(int(r['Calls']) for r in rows)} launches")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    n = r["Name"].replace("(anonymous namespace)::", "")
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}% {int(r['Calls']):7d} "
          f"{float(r['AverageNs']) / 1e3:9.1f}us  {n[:110]}")
