"""PINN train steps (configs[3], B=64, 64x64) for rocprofv3: the graph-mode step as the bench
runs it (one eager step + one counted eager step, the capture, then the timed replays).
argv[1] = "eager" times the eager step instead."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
from dist import DistContext  # noqa: E402


class A:
    pass


args = A()
args.batch = None
args.weak = False
args.per_rank_of = None
args.pinn_warmup = 2
args.pinn_steps = 5
args.pinn_eager = len(sys.argv) > 1 and sys.argv[1] == "eager"
dev = torch.device("cuda:0")
print(bench.bench_pinn(args, DistContext(), dev), flush=True)
