"""upfirdn2d up2 (NCSN++ FIR upsample, k=[1,3,3,1] x gain 4, pad (2,1)) timing on the
sampler shapes; prints ms per launch and GB/s (4 * (in + out) bytes)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import numpy as np
import torch
from op import upfirdn2d
dev = torch.device("cuda:0")
k = torch.tensor(np.outer([1, 3, 3, 1], [1, 3, 3, 1]) / 64.0 * 4, dtype=torch.float32, device=dev)
for shape in [(64, 256, 64, 64), (64, 256, 32, 32), (64, 128, 64, 64)]:
    x = torch.randn(*shape, device=dev)
    for _ in range(3):
        y = upfirdn2d(x, k, up=2, pad=(2, 1))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        y = upfirdn2d(x, k, up=2, pad=(2, 1))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    gb = 4 * (x.numel() + y.numel()) / 1e9
    print(shape, f"{ms:.4f} ms", f"{gb / ms * 1e3:.0f} GB/s", flush=True)
