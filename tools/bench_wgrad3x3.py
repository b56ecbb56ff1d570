"""Winograd 3x3 weight gradient (split-K + reduce) on the PINN's shapes (configs[3]) at B = 8 and
64 and a few NCSN++ shapes: us per call vs an fp64 reference (BPK_LIB selects the library)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
from op import _hipenv  # noqa: E402,F401
import torch  # noqa: E402

from op.conv import conv3x3_wgrad_raw  # noqa: E402

SHAPES = [(128, 16, 64), (192, 96, 32), (64, 32, 64), (64, 16, 64), (320, 160, 16), (192, 32, 32),
          (32, 16, 64), (32, 32, 64), (64, 32, 32), (448, 224, 8), (128, 128, 128), (256, 256, 16)]
dev = torch.device("cuda:0")
tot = {}
for B in (8, 64):
    t_all = 0.0
    for cin, cout, hw in SHAPES:
        if B == 64 and hw == 128:
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(B, cin, hw, hw, device=dev, generator=g)
        gy = torch.randn(B, cout, hw, hw, device=dev, generator=g)
        ws = (cout, cin, 3, 3)
        dw, db = conv3x3_wgrad_raw(x, gy, ws, bias_grad=True)
        ref = torch.nn.grad.conv2d_weight(x.double(), ws, gy.double(), padding=1)
        err = ((dw.double() - ref).abs().max() / ref.abs().max()).item()
        for _ in range(3):
            conv3x3_wgrad_raw(x, gy, ws, bias_grad=True)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            conv3x3_wgrad_raw(x, gy, ws, bias_grad=True)
        e.record()
        e.synchronize()
        us = s.elapsed_time(e) / 10 * 1e3
        t_all += us
        print(json.dumps({"B": B, "shape": f"{cin}->{cout}@{hw}", "us": round(us, 1), "err": float(f"{err:.1e}")}))
    tot[B] = round(t_all, 1)
print(json.dumps({"summary": "sum of us over the shapes", "lib": os.environ.get("BPK_LIB", "default"), "total_us": tot}))
