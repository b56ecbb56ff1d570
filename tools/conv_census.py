"""Which Winograd conv forms one NCSN++ 128x128 score-net forward launches (the bench model, B=64,
inference): counts of bpk_conv3x3_wino_ex_f32 calls by (GroupNorm prologue, residual tail,
two sources, shape).  Diagnostic for the sampler's kernel mix."""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
from op._lib import lib  # noqa: E402

dev = torch.device("cuda:0")
c, model = bench.build_model(dev)
model.eval()
fn = lib.bpk_conv3x3_wino_ex_f32
calls = collections.Counter()


def wrapped(x, x2, C1, pre, U, bias, skip, div, y, stats, N, Cin, Cout, H, W, stream):
    calls[(pre is not None, skip is not None, x2 is not None, stats is not None,
           f"{Cin}->{Cout}@{H}")] += 1
    return fn(x, x2, C1, pre, U, bias, skip, div, y, stats, N, Cin, Cout, H, W, stream)


lib.bpk_conv3x3_wino_ex_f32 = wrapped
x = torch.randn(64, 1, 128, 128, device=dev)
t = torch.rand(64, device=dev) * 999
with torch.no_grad():
    model(x, t)
    calls.clear()
    model(x, t)
torch.cuda.synchronize()
print("pre skip x2 stats shape: calls per forward")
for k, v in sorted(calls.items(), key=lambda kv: (-kv[1], kv[0])):
    print(k, v)
