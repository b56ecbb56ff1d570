"""PINN step losses per step, eager vs hipGraph replay (bench's configs[3] setup):
usage python tools/diag_pinn_graph.py [steps]"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
import bench
import losses
from configs.pinn import pinn_pde
from dist import DistContext
from inverse.operators import get_operator
from models.ema import ExponentialMovingAverage
from pinn_kalman.pinn import PINN

dev = torch.device("cuda:0")
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
frozen = os.environ.get("DIAG_FROZEN") == "1"
if os.environ.get("DIAG_NORNG") == "1":  # observation without the randn draw
    losses._observe = lambda config, operator, f: operator(f, keep_shape=True)  # lr 0 and no observation noise: every step identical
for graph in ((True,) if frozen else (False, True)):
    c = pinn_pde.get_config()
    c.device = dev
    if frozen:
        c.optim.lr = 0.0
        c.inverse.variance = 0.0
    torch.manual_seed(0)
    model = PINN(c)
    ema = ExponentialMovingAverage(model.parameters(), decay=c.model.ema_rate)
    opt_f = losses.get_optimizer(c, model.flownet.parameters())
    opt_p = losses.get_optimizer(c, model.pressurenet.parameters(), 0.005)
    state = dict(optimizer=(opt_f, opt_p), model=model, ema=ema, step=c.training.n_iters)
    opt_fn = losses.optimization_manager(c)
    if os.environ.get("DIAG_NOOPT") == "1":
        opt_fn = lambda *a, **k: None
    step_fn = losses.get_pinn_step_fn(c, train=True, optimize_fn=opt_fn,
                                      ctx=DistContext(), graph=graph)
    operator = get_operator(c)
    if os.environ.get("DIAG_FIXMASK") == "1":
        from inverse.operators import InpaintOperator
        operator = InpaintOperator(mask=[operator.mask])
    batch = bench.pinn_batch(c, 64, dev, seed=0)
    for i in range(steps):
        out = step_fn(state, operator, batch)
        gn = sum(float(p.grad.norm()) ** 2 for p in model.parameters() if p.grad is not None) ** 0.5
        print("graph" if graph else "eager", i, [round(float(v), 6) for v in out], "gradnorm", round(gn, 4), flush=True)
