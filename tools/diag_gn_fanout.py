"""Which gradient of a training-mode BigGAN up block differs with the GroupNorm fan-out, and
is the block run-to-run deterministic without it (diagnostic)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
from op import _hipenv  # noqa
import torch
from models import layers
from models import layerspp as lpp
hip = torch.device("cuda:0")
torch.manual_seed(2)
blk = lpp.ResnetBlockBigGANpp(act=torch.nn.SiLU(), in_ch=64, out_ch=64, temb_dim=32, up=True,
                              fir=True, dropout=0.0, skip_rescale=True).to(hip).train()
x0 = torch.randn(4, 64, 16, 16, device=hip)
temb = torch.randn(4, 32, device=hip)
def grads(fan):
    layers._GN_FANOUT = fan
    blk.zero_grad(set_to_none=True)
    x = x0.clone().requires_grad_()
    y = blk(x * 1.0, temb)
    (y * torch.linspace(-1, 1, y.numel(), device=hip).view_as(y)).sum().backward()
    return [("y", y.detach()), ("x", x.grad)] + [(n, p.grad.clone()) for n, p in blk.named_parameters()]
a1, a2, b1, b2 = grads(True), grads(True), grads(False), grads(False)
for (n, t1), (_, t2), (_, u1), (_, u2) in zip(a1, a2, b1, b2):
    print(f"{n:24s} fan-fan {float((t1-t2).abs().max()):.3e}  plain-plain {float((u1-u2).abs().max()):.3e}  fan-plain {float((t1-u1).abs().max()):.3e}")
