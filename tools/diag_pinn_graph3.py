"""diag_pinn_graph2 made step_fn-like, with toggles (env DIAG_T = subset of 'obs,copy,nan,ema,static')
to find what makes the PINN hipGraph replay read stale memory after a few replays."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
import bench
from configs.pinn import pinn_pde
from models.ema import ExponentialMovingAverage
from pinn_kalman.pinn import PINN

T = set(os.environ.get("DIAG_T", "").split(","))
dev = torch.device("cuda:0")
c = pinn_pde.get_config()
c.device = dev
torch.manual_seed(0)
model = PINN(c).train()
ema = ExponentialMovingAverage(model.parameters(), decay=c.model.ema_rate)
batch = bench.pinn_batch(c, 64, dev, seed=0)
if "static" in T:
    sb = tuple(v.detach().clone().requires_grad_(v.requires_grad) for v in batch)
else:
    sb = tuple(v.detach().clone() for v in batch[:2]) + tuple(
        v.detach().clone().requires_grad_() for v in batch[2:5]) + (batch[5],)
mask = (torch.rand(64, 1, 64, 64, device=dev) > 0.1).float()
params = [p for p in model.parameters() if p.requires_grad]


def loss_fn():
    f1, f2, x, y, t, target = sb
    if "obs" in T:
        f1, f2 = mask * f1, mask * f2
    flows, pres = model(f1, f2, x, y, t)
    data = model.flownet.multiscale_data_mse(flows, target) + model.pressurenet.data_mse(pres, target)
    pl = model.equation_mse(x, y, t, flows[-1], pres, 10000000.0) * c.training.pinn_loss_weight
    return pl + data, pl, data


for i in range(2):  # eager steps
    model.zero_grad(set_to_none=True)
    l = loss_fn()
    l[0].backward()
    print("eager", i, [float(v) for v in l], flush=True)
side = torch.cuda.Stream(dev)
side.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(side):
    model.zero_grad(set_to_none=True)
    w = loss_fn()
    w[0].backward()
    del w
torch.cuda.current_stream(dev).wait_stream(side)
model.zero_grad(set_to_none=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out = loss_fn()
    for p in params:
        if p.grad is not None:
            p.grad.zero_()
    out[0].backward()
out = [o.detach() for o in out]
for i in range(10):
    if "copy" in T:
        with torch.no_grad():
            for s_, v in zip(sb, batch):
                s_.copy_(v)
    g.replay()
    if "nan" in T:
        bad = bool(torch.isnan(model.pressurenet.end[-1].weight.grad).any())
    if "ema" in T:
        ema.update(model.parameters())
    print("replay", i, [float(o) for o in out], flush=True)
