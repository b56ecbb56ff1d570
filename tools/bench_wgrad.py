"""Winograd weight gradient vs MIOpen backward-weights on the NCSN++ shapes: error + time."""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
from op.conv import conv3x3_wgrad_raw
dev = torch.device("cuda:0")
B = int(os.environ.get("B", 64))
shapes = [(128, 128, 128), (256, 128, 128), (256, 256, 128), (256, 256, 64), (512, 256, 64),
          (256, 256, 32), (512, 256, 32), (256, 256, 16), (128, 256, 64)]
def t_of(fn, reps=10):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / reps / 1e3
for cin, cout, hw in shapes:
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, cin, hw, hw, device=dev, generator=g)
    gy = torch.randn(B, cout, hw, hw, device=dev, generator=g)
    ws = (cout, cin, 3, 3)
    ref = torch.nn.grad.conv2d_weight(x, ws, gy, padding=1)
    out = conv3x3_wgrad_raw(x, gy, ws)
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    tw = t_of(lambda: conv3x3_wgrad_raw(x, gy, ws))
    tm = t_of(lambda: torch.nn.grad.conv2d_weight(x, ws, gy, padding=1))
    fl = 2.0 * B * cin * cout * 9 * hw * hw
    print(json.dumps(dict(shape=f"{cin}->{cout}@{hw}", rel_err_vs_miopen=float(f"{err:.2e}"),
                          wino_ms=round(tw * 1e3, 3), miopen_ms=round(tm * 1e3, 3),
                          wino_tflops_eff=round(fl / tw / 1e12, 1),
                          miopen_tflops=round(fl / tm / 1e12, 1))), flush=True)
