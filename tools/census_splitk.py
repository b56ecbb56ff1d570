"""Census of the split-K launches of one PINN train step (configs[3]) at a per-rank batch:
every implicit-GEMM / Winograd weight-gradient / 1x1 weight-gradient call with its shape, so
the split counts (and with them the separate reduce launches) can be recomputed on the host.

    python tools/census_splitk.py [per-rank-of N] > out.json

Runs the eager step (the graph step replays the same calls)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
from op import _hipenv  # noqa: E402,F401
import torch  # noqa: E402

import bench  # noqa: E402
from dist import DistContext  # noqa: E402
from op._lib import lib  # noqa: E402

LOG = []
RECORD = [False]
NAMES = {
    "bpk_conv2d_igemm_fwd_f32": (5, 19), "bpk_conv2d_igemm_dgrad_f32": (4, 18),
    "bpk_conv2d_igemm_wgrad_f32": (5, 19), "bpk_conv3x3_wino_wgrad_f32": (4, 9),
    "bpk_conv3x3_wino_wgrad_bias_f32": (5, 10), "bpk_conv3x3_wino_wgrad_pre_f32": (6, 11),
    "bpk_gemm_nchw_wgrad_f32": (4, 8), "bpk_conv2d_wgrad_small_cout_f32": (5, 11),
}


def wrap(name, lo, hi):
    dll = lib.load()
    fn = getattr(dll, name)

    def w(*a):
        if RECORD[0]:
            LOG.append([name] + [int(v) if isinstance(v, int) else None for v in a[lo:hi]]
                       + [a[3] is not None if "igemm_wgrad" in name else None])
        return fn(*a)
    setattr(dll, name, w)


for k, (lo, hi) in NAMES.items():
    wrap(k, lo, hi)


class A:
    pass


args = A()
args.batch = None
args.weak = False
args.per_rank_of = int(sys.argv[1]) if len(sys.argv) > 1 else 8
args.pinn_warmup = 2
args.pinn_steps = 1
args.pinn_eager = True
dev = torch.device("cuda:0")
bench.bench_pinn(args, DistContext(), dev)
RECORD[0] = True
args.pinn_warmup = 0
bench.bench_pinn(args, DistContext(), dev)
json.dump(LOG, sys.stdout)
