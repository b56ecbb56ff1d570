"""Dominant-kernel launches for the HBM-traffic PMC passes (rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE, one counter per pass): 10 x Winograd conv3x3 128->128 @128^2 B=64 (the bench
roofline kernel) and 10 x upfirdn2d down2 [64,128,128,128]."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import numpy as np
import torch
from op import upfirdn2d
from op.conv import conv3x3, filter_transform
dev = torch.device("cuda:0")
x = torch.randn(64, 128, 128, 128, device=dev)
w = torch.randn(128, 128, 3, 3, device=dev) * 0.02
filter_transform(w)
for _ in range(10):
    conv3x3(x, w)
k = torch.tensor(np.outer([1, 3, 3, 1], [1, 3, 3, 1]) / 64.0, dtype=torch.float32, device=dev)
for _ in range(10):
    upfirdn2d(x, k, down=2, pad=(1, 1))
torch.cuda.synchronize()
print("ok")
