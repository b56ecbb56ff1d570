"""PINN train steps (configs[3], 64x64) for rocprofv3: the graph-mode step as the bench runs it
(the capture, then the timed replays, then one counted eager step).

    python tools/prof_pinn.py [eager|graph] [per-rank-of N] [steps]

"eager" times the eager step; the per-rank batch is 64 / N (N = 8: the per-rank work of the
8-GPU point, B = 8)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
from op import _hipenv  # noqa: E402,F401  (before torch touches the device)
import torch  # noqa: E402

import bench  # noqa: E402
from dist import DistContext  # noqa: E402


class A:
    pass


argv = sys.argv[1:]
args = A()
args.batch = None
args.weak = False
args.per_rank_of = int(argv[1]) if len(argv) > 1 else None
args.pinn_warmup = 2
args.pinn_steps = int(argv[2]) if len(argv) > 2 else 5
args.pinn_eager = len(argv) > 0 and argv[0] == "eager"
dev = torch.device("cuda:0")
print(bench.bench_pinn(args, DistContext(), dev), flush=True)
