"""20 launches of the Winograd conv3x3 on 128->128 @128^2, B=64 (for rocprofv3 counters)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
from op.conv import conv3x3
dev = torch.device("cuda:0")
x = torch.randn(64, 128, 128, 128, device=dev)
w = torch.randn(128, 128, 3, 3, device=dev) * 0.02
for _ in range(20):
    y = conv3x3(x, w)
torch.cuda.synchronize()
print("ok")
