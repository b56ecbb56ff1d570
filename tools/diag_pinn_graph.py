"""Diagnostic: the bench's PINN phase (configs[3], B = 64, random masks, variance 0.01) with
the eager step and the hipGraph step from the same state and seeds; prints the three losses
of each step for both and whether the graph's static inputs / outputs are finite."""
import copy
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import losses  # noqa: E402
from configs.pinn import pinn_pde  # noqa: E402
from inverse.operators import get_operator  # noqa: E402
from models.ema import ExponentialMovingAverage  # noqa: E402
from pinn_kalman.pinn import PINN  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
c = pinn_pde.get_config()
c.device = dev
c.training.batch_size = B
torch.manual_seed(0)
m0 = PINN(c)
batch = bench.pinn_batch(c, B, dev)
masks = get_operator(c).params["mask"]

for graph in (False, True):
    m = copy.deepcopy(m0).to(dev)
    ema = ExponentialMovingAverage(m.parameters(), decay=c.model.ema_rate)
    state = dict(optimizer=(losses.get_optimizer(c, m.flownet.parameters()),
                            losses.get_optimizer(c, m.pressurenet.parameters(), 0.005)),
                 model=m, ema=ema, step=c.training.n_iters)
    fn = losses.get_pinn_step_fn(c, train=True, graph=graph,
                                 optimize_fn=losses.optimization_manager(c))
    from inverse.operators import InpaintOperator
    op = InpaintOperator(mask=masks)
    torch.manual_seed(7)
    for i in range(4):
        out = fn(state, op, batch)
        print("graph" if graph else "eager", i, [round(float(v), 6) for v in out], flush=True)
    if graph:
        print("static finite", [bool(torch.isfinite(t).all()) for t in fn.static],
              "noise", [float(z.abs().max()) for z in fn.noise],
              "mask", float(fn.mask.sum()), flush=True)
