import os, sys
REPO = "/root/repo"
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch, torch.nn.functional as F
from op.conv import conv3x3
dev = torch.device("cuda:0")
for (N, cin, cout, hw) in [(1, 16, 128, 32), (2, 32, 64, 32), (1, 16, 256, 16), (3, 48, 128, 64), (64, 16, 128, 32)]:
    x = torch.randn(N, cin, hw, hw, device=dev)
    w = torch.randn(cout, cin, 3, 3, device=dev)
    out = conv3x3(x, w); ref = F.conv2d(x, w, padding=1)
    e = (out - ref).abs()
    bad = (e > 1e-3 * ref.abs().max())
    print(N, cin, cout, hw, float(e.max()), int(bad.sum()), bad.nonzero()[:3].tolist() if bad.any() else None)
