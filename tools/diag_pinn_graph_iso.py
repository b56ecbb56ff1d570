"""Diagnostic: the captured PINN step replayed with the parameters fixed (no optimizer, no
EMA, noise buffers fixed) -- every replay must give the same losses.  argv[1]: "plain"
(replays only) | "churn" (eager allocations of assorted sizes between replays) | "opt"
(the optimizer step between replays, losses compared with eager steps elsewhere)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import losses  # noqa: E402
from configs.pinn import pinn_pde  # noqa: E402
from inverse.operators import get_operator  # noqa: E402
from pinn_kalman.pinn import PINN  # noqa: E402

mode = sys.argv[1]
dev = torch.device("cuda:0")
c = pinn_pde.get_config()
c.device = dev
c.training.batch_size = 64
torch.manual_seed(0)
model = PINN(c)
model.train()
fn = losses.get_pinn_step_fn(c, train=True, optimize_fn=losses.optimization_manager(c),
                             graph=True)
operator = get_operator(c)
operator.next()
batch = bench.pinn_batch(c, 64, dev, seed=0)
fn._capture(model, operator, batch)
if "nofill" not in mode:
    with torch.no_grad():
        for d, b in zip(fn.static, batch):
            d.copy_(b)
        fn.mask.copy_(operator.mask.to(dev))
        for z in fn.noise:
            z.normal_()
keep = []
for i in range(16):
    fn.graph.replay()
    vals = [float(t) for t in fn.out]
    gsum = 0.0 if "nogsum" in mode else float(sum(
        p.grad.double().abs().sum() for p in model.parameters() if p.grad is not None))
    print(mode.split("-")[0], i, [round(v, 6) for v in vals], "gradsum", round(gsum, 6), flush=True)
    if mode.startswith("redunrel"):  # eager reductions of tensors the graph never sees
        for k in range(1, 40):
            float(torch.randn((k * 7919) % 300000 + 1, device=dev).double().abs().sum())
    if mode.startswith("churn"):
        for k in range(1, 40):
            keep.append(torch.randn((k * 7919) % 300000 + 1, device=dev))
        if len(keep) > 200:
            del keep[:100]
