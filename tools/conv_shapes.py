"""Per-shape MIOpen fp32 conv throughput for the NCSN++ 128^2 conv inventory (B = 64)."""
import json, os, sys, time
import torch
import torch.nn.functional as F
dev = torch.device("cuda:0")
B = int(os.environ.get("B", 64))
shapes = [  # (cin, cout, hw, k, count per fwd)
    (128, 128, 128, 3, 13), (256, 128, 128, 3, 4), (256, 256, 128, 3, 2), (384, 128, 128, 3, 0),
    (256, 256, 64, 3, 14), (512, 256, 64, 3, 4), (256, 256, 32, 3, 17), (512, 256, 32, 3, 0),
    (256, 256, 16, 3, 0), (128, 256, 64, 3, 1), (1, 128, 128, 3, 1), (128, 1, 128, 3, 1)]
res = []
for cin, cout, hw, k, cnt in shapes:
    x = torch.randn(B, cin, hw, hw, device=dev)
    w = torch.randn(cout, cin, k, k, device=dev) * 0.02
    for _ in range(3):
        F.conv2d(x, w, padding=k // 2)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        F.conv2d(x, w, padding=k // 2)
    e.record(); e.synchronize()
    t = s.elapsed_time(e) / 10 / 1e3
    fl = 2.0 * B * cout * cin * k * k * hw * hw
    res.append(dict(shape=f"{cin}->{cout}@{hw}", ms=round(t * 1e3, 3), tflops=round(fl / t / 1e12, 1),
                    per_fwd=cnt))
    print(json.dumps(res[-1]), flush=True)
