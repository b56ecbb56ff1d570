"""Weighted PRE-conv mix time from a rocprofv3 kernel trace of tools/bench_wino_mix.py:
per shape, the mean duration of the wino_f23_pipe_kernel<1, true, 8 | 4> launches of its PRE+stats
and PRE+residual runs (3 warm-up + REPS each, in launch order), weighted by the per-forward
counts of bench_wino_mix.MIX -- to compare with the HIP-event figure the bench prints.
usage: roofline_mix_from_trace.py kernel_trace.csv [REPS]"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_wino_mix import MIX  # noqa: E402

reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rows = sorted((r for r in csv.DictReader(open(sys.argv[1]))
               if "wino_f23_pipe_kernel<1, true," in r["Kernel_Name"]),
              key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
per = 3 + reps
assert len(dur) == 2 * per * len(MIX), (len(dur), 2 * per * len(MIX))
tot_ms = tot_f = 0.0
shapes = []
for i, (cin, cout, hw, n_pre, n_res) in enumerate(MIX):
    pre = dur[2 * i * per + 3: 2 * i * per + per]
    res = dur[(2 * i + 1) * per + 3: (2 * i + 2) * per]
    t_pre, t_res = sum(pre) / len(pre), sum(res) / len(res)
    fl = 2.0 * 64 * cin * cout * 16 * (hw // 2) ** 2
    tot_ms += n_pre * t_pre + n_res * t_res
    tot_f += (n_pre + n_res) * fl
    shapes.append(dict(shape=f"{cin}->{cout}@{hw}", pre_ms=round(t_pre, 4), res_ms=round(t_res, 4)))
print(json.dumps(dict(source="rocprofv3 kernel trace", ms_per_forward_mix=round(tot_ms, 3),
                      tflops_executed=round(tot_f / tot_ms / 1e9, 2),
                      frac_of_157_3=round(tot_f / tot_ms / 1e9 / 157.3, 4), per_shape=shapes)))
