"""Diagnostic: the bench's PINN phase sequence on one state -- eager step, eager step under
op.flops counting (argv[1] = "nocount": a plain eager step instead; "noeager": neither),
then 12 hipGraph steps -- printing each step's three losses."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import losses  # noqa: E402
from configs.pinn import pinn_pde  # noqa: E402
from dist import DistContext  # noqa: E402
from inverse.operators import get_operator  # noqa: E402
from models.ema import ExponentialMovingAverage  # noqa: E402
from pinn_kalman.pinn import PINN  # noqa: E402

variant = sys.argv[1] if len(sys.argv) > 1 else "bench"
# "eager12": 12 eager steps instead of the graph steps (same seeds: numerics vs capture)
dev = torch.device("cuda:0")
ctx = DistContext()
c = pinn_pde.get_config()
c.device = dev
torch.manual_seed(0)
model = PINN(c)
ema = ExponentialMovingAverage(model.parameters(), decay=c.model.ema_rate)
state = dict(optimizer=(losses.get_optimizer(c, model.flownet.parameters()),
                        losses.get_optimizer(c, model.pressurenet.parameters(), 0.005)),
             model=model, ema=ema, step=c.training.n_iters)
eager_fn = losses.get_pinn_step_fn(c, train=True, optimize_fn=losses.optimization_manager(c),
                                   ctx=ctx)
graph_fn = losses.get_pinn_step_fn(c, train=True, optimize_fn=losses.optimization_manager(c),
                                   ctx=ctx, graph=True)
B = 64
c.training.batch_size = B
operator = get_operator(c)
batch = bench.pinn_batch(c, B, dev, seed=0)
if variant not in ("noeager", "eager12"):
    print("eager a", [round(float(v), 6) for v in eager_fn(state, operator, batch)], flush=True)
    if variant == "nocount":
        out = eager_fn(state, operator, batch)
    else:
        _, out = bench.counted(lambda: eager_fn(state, operator, batch), dev)
    print("eager b", [round(float(v), 6) for v in out], flush=True)
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
for i in range(steps):
    fn = eager_fn if variant == "eager12" else graph_fn
    out = fn(state, operator, batch)
    print(variant, i, [round(float(v), 6) for v in out], flush=True)
