"""Where the PINN graph step's kernels go, by phase: a marker kernel (torch.cuda._sleep) is
recorded between the phases of the captured step (forward, the three first-order derivative
passes, the four second-order passes, the residual, the final backward); run under rocprofv3
--kernel-trace and split the trace at the markers with `--split TRACE.csv`.

    python tools/prof_pinn_phases.py [per-rank-of N]
    python tools/prof_pinn_phases.py --split TRACE.csv"""
import collections
import csv
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO, os.path.join(REPO, "tools")]

# the residual's derivative passes: the reference's seven (BPK_PINN_COPIES=1) or batched over
# input copies (PINN.forward_residual_copies: one first-order pass, one / two second-order)
PHASES = (["forward", "d1_u", "d1_v", "d1_p", "d2", "residual", "backward"]
          if os.environ.get("BPK_PINN_COPIES") == "1" else
          ["forward", "d1", "d2", "residual", "backward"])

if len(sys.argv) > 2 and sys.argv[1] == "--split":
    import re

    def short(n):  # as tools/trace_steps.py
        n = n.replace("(anonymous namespace)::", "")
        if "at::native" in n:
            m = re.search(r"at::native::(?:\(anonymous namespace\)::)?(\w+)<[^,]*,\s*at::native::([\w:]+)", n)
            return "aten:" + (m.group(2) if m else n[:60])
        return n.split("(")[0][:70]
    rows = list(csv.DictReader(open(sys.argv[2])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    marks = [i for i, e in enumerate(ev) if "sleep" in e[2].lower() or "spin" in e[2].lower()]
    # the last replay's markers: the step runs forward .. backward, then the copies / graph B
    last = marks[-len(PHASES):]
    ends = last[1:] + [None]
    for name, a, b in zip(PHASES, last, ends):
        seg = ev[a + 1:b] if b is not None else ev[a + 1:a + 1 + 4000]
        if b is None:  # until the first gap > 1 ms (end of the replay)
            for j in range(1, len(seg)):
                if seg[j][0] - seg[j - 1][1] > 1_000_000:
                    seg = seg[:j]
                    break
        busy = sum(e[1] - e[0] for e in seg) / 1e6
        span = (seg[-1][1] - seg[0][0]) / 1e6 if seg else 0.0
        c = collections.Counter(short(e[2]) for e in seg)
        aten = sum(v for k, v in c.items() if k.startswith("aten"))
        print(f"{name:9s} {len(seg):5d} kernels ({aten:4d} aten)  busy {busy:6.2f} ms  span {span:6.2f} ms")
        print("          " + ", ".join(f"{k[:40]} {v}" for k, v in c.most_common(8)))
    sys.exit(0)

from op import _hipenv  # noqa: E402,F401
import torch  # noqa: E402

import bench  # noqa: E402
from dist import DistContext  # noqa: E402
from pinn_kalman import pinn  # noqa: E402

pinn.PHASE_MARK = lambda name: torch.cuda._sleep(100)


class A:
    pass


args = A()
args.batch = None
args.weak = False
args.per_rank_of = int(sys.argv[1]) if len(sys.argv) > 1 else None
args.pinn_warmup = 2
args.pinn_steps = 3
args.pinn_eager = False
dev = torch.device("cuda:0")
dt, losses_, tally, B = bench._pinn_run(args, DistContext(), dev)
print({"B": B, "ms_per_step": dt / args.pinn_steps * 1e3, "losses": losses_}, flush=True)
