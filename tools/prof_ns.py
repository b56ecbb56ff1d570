"""ns_step kernels under rocprofv3: 20 fused full steps + 20 three-op steps (B256 192^2)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
from op import ns_step
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
B, n = 256, 192
f = torch.rand(B, 1, n, n, device=dev, generator=g) * 0.9 + 0.1
p = torch.randn(B, 1, n, n, device=dev, generator=g) * 0.01
v = (torch.rand(B, 2, n, n, device=dev, generator=g) * 0.45 + 0.05) * \
    torch.sign(torch.randn(B, 2, n, n, device=dev, generator=g))
for _ in range(20):
    ns_step.full_step(f, v, p, 0.0025, 0.005)
for _ in range(20):
    v1 = ns_step.update_velocity(v, p, 0.0025, 0.005)
    p1 = ns_step.update_pressure(p, v1, 0.0025, 0.005)
    f1 = ns_step.update_density(f, v1, 0.0025, 0.005)
torch.cuda.synchronize()
print("done")
