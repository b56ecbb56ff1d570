"""Diagnostic: which part of the captured PINN step reads memory it does not own.  Captures
one piece of the step (argv[1]): "fwd" (observation + both nets + data loss), "res" (+ the
residual's autograd derivatives, no backward), "full" (+ backward w.r.t. the parameters);
replays it 12 times with fixed inputs and eager allocations in between; prints the outputs."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import losses  # noqa: E402
from configs.pinn import pinn_pde  # noqa: E402
from op import conv as conv_op  # noqa: E402
from pinn_kalman.pinn import PINN  # noqa: E402

mode = sys.argv[1]
dev = torch.device("cuda:0")
c = pinn_pde.get_config()
c.device = dev
torch.manual_seed(0)
model = PINN(c)
model.train()
params = list(model.parameters())
batch = [b.detach().clone() for b in bench.pinn_batch(c, 64, dev, seed=0)]
for i in (2, 3, 4):
    batch[i].requires_grad_(True)
mask = (torch.rand(64, 1, 64, 64, device=dev) > 0.5).float()
noise = (torch.randn_like(batch[0]), torch.randn_like(batch[1]))
sop = losses._MaskOperator(mask)


def piece():
    f1, f2, x, y, t, target = batch
    f1 = losses._observe(c, sop, f1, noise[0])
    f2 = losses._observe(c, sop, f2, noise[1])
    flow_pred, pres_pred = model(f1, f2, x, y, t)
    data_loss = (model.flownet.multiscale_data_mse(flow_pred, target)
                 + model.pressurenet.data_mse(pres_pred, target))
    if mode == "lossfn":  # the step's own loss function, outputs as _PinnGraphStep keeps them
        loss, pl, dl = LOSS_FN(model, sop, batch, noise)
        loss.backward(inputs=params)
        return (loss, pl, dl)
    if mode == "fwd":
        return (data_loss, flow_pred[-1].sum(), pres_pred.sum())
    pinn = model.equation_mse(x, y, t, flow_pred[-1], pres_pred, 10000000.0)
    if mode == "res":
        return (data_loss, pinn, flow_pred[-1].sum())
    loss = pinn * c.training.pinn_loss_weight + data_loss
    loss.backward(inputs=params)
    if mode == "fullkeep":  # the loss tensor (and with it the captured autograd graph) kept
        return (data_loss, pinn, loss)
    return (data_loss, pinn, sum(p.grad.sum() for p in params if p.grad is not None))


LOSS_FN = losses.get_pinn_step_fn(c, train=True, optimize_fn=None, graph=True).loss_fn
with conv_op.native_only():
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(2):
            for p in params:
                p.grad = None
            ref = [float(v) for v in piece()]
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize(dev)
    for p in params:
        p.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out = piece()
print(mode, "eager", [round(v, 6) for v in ref], flush=True)
keep = []
for i in range(12):
    g.replay()
    print(mode, i, [round(float(v), 6) for v in out], flush=True)
    for k in range(1, 40):
        keep.append(torch.randn((k * 7919) % 300000 + 1, device=dev))
    if len(keep) > 200:
        del keep[:100]
