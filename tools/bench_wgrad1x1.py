"""1x1-conv weight gradient (gemm_nchw_wgrad, split-K + reduce) on PressureNet's shortcut
shapes (configs[3]) at B = 8 and 64: us per call (BPK_LIB selects the library)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
from op import _hipenv  # noqa: E402,F401
import torch  # noqa: E402

from op.conv import _wgrad1x1_raw  # noqa: E402

SHAPES = [(32, 64, 64), (64, 16, 64), (64, 128, 64), (128, 16, 64), (16, 32, 32), (96, 192, 32),
          (192, 32, 32), (32, 64, 16), (160, 320, 16), (320, 64, 16), (64, 128, 8), (224, 448, 8),
          (448, 96, 8), (96, 192, 4)]
dev = torch.device("cuda:0")
tot = {}
for B in (8, 64):
    t_all = 0.0
    for cin, cout, hw in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(B, cin, hw, hw, device=dev, generator=g)
        gy = torch.randn(B, cout, hw, hw, device=dev, generator=g)
        ref = torch.einsum("nmp,nkp->mk", gy.flatten(2).double(), x.flatten(2).double())
        dw, db = _wgrad1x1_raw(gy, x, True)
        err = ((dw.double() - ref).abs().max() / ref.abs().max()).item()
        for _ in range(3):
            _wgrad1x1_raw(gy, x, True)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            _wgrad1x1_raw(gy, x, True)
        e.record()
        e.synchronize()
        us = s.elapsed_time(e) / 20 * 1e3
        t_all += us
        print(json.dumps({"B": B, "shape": f"{cin}->{cout}@{hw}", "us": round(us, 1), "err": float(f"{err:.1e}")}))
    tot[B] = round(t_all, 1)
print(json.dumps({"summary": "sum of us over the shapes", "lib": os.environ.get("BPK_LIB", "default"), "total_us": tot}))
