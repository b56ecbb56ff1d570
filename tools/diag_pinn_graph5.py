"""(DIAG5 toggles) The bench's PINN step (bench._pinn_run setup: pinn_pde B=64, bench.pinn_batch, the 1600
random inpainting masks, observation noise) eager vs get_pinn_step_fn(graph=True), losses of
every step, with toggles (env DIAG): var0 = observation variance 0, mask1 = one fixed mask,
block = blocking mask copy."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import losses  # noqa: E402
from configs.pinn import pinn_pde  # noqa: E402
from inverse.operators import InpaintOperator, get_operator  # noqa: E402
from models.ema import ExponentialMovingAverage  # noqa: E402
from pinn_kalman.pinn import PINN  # noqa: E402

T = set(os.environ.get("DIAG5", "").split(","))
dev = torch.device("cuda:0")


def run(graph, steps=int(os.environ.get("DIAG_STEPS", 12))):
    c = pinn_pde.get_config()
    c.device = dev
    if "var0" in T:
        c.inverse.variance = 0.0
    torch.manual_seed(0)
    model = PINN(c)
    ema = ExponentialMovingAverage(model.parameters(), decay=c.model.ema_rate)
    opt_f = losses.get_optimizer(c, model.flownet.parameters())
    opt_p = losses.get_optimizer(c, model.pressurenet.parameters(), 0.005)
    state = dict(optimizer=(opt_f, opt_p), model=model, ema=ema, step=c.training.n_iters)
    opt_fn = losses.optimization_manager(c)
    if "noopt" in T:  # parameters fixed: every step the same forward / backward
        opt_fn = lambda *a, **k: None  # noqa: E731
    if "sync" in T:
        real = opt_fn

        def opt_fn(*a, _r=real, **k):
            torch.cuda.synchronize()
            return _r(*a, **k)
    step_fn = losses.get_pinn_step_fn(c, train=True, optimize_fn=opt_fn, graph=graph)
    if "mask1" in T:
        g = torch.Generator().manual_seed(3)
        operator = InpaintOperator(mask=[(torch.rand(64, 1, 64, 64, generator=g) > 0.1).float()])
    else:
        torch.manual_seed(1)
        operator = get_operator(c)
    batch = bench.pinn_batch(c, 64, dev, seed=0)
    torch.manual_seed(2)
    out = []
    for _ in range(steps):
        lo = step_fn(state, operator, batch)
        out.append([round(float(v), 5) for v in lo])
    return out


if "block" in T:
    _orig = torch.Tensor.copy_

    def _copy(self, src, non_blocking=False):
        return _orig(self, src, False)
    torch.Tensor.copy_ = _copy

e = run(False)
g = run(True)
print("DIAG", sorted(T))
for i, (a, b) in enumerate(zip(e, g)):
    print(i, "eager", a, "graph", b, flush=True)
