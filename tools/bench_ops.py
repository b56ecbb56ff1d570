"""Micro-benchmarks of the hand-written HBM-bound kernels at the NCSN++ 128^2 B=64 shapes
(BASELINE.md "upfirdn2d" shapes; GroupNorm+SiLU; residual).  GB/s = algorithmic bytes / time."""
import json
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "b-pinn-kalman-filter_amd")]
import numpy as np
import torch

from op import upfirdn2d
from op.norm_act import group_norm_act_f, residual_rescale


def t_of(fn, reps=20):
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    for _ in range(3):
        fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / 1e3 / reps


dev = "cuda"
res = {}
k = torch.tensor(np.outer([1, 3, 3, 1], [1, 3, 3, 1]) / 64.0, dtype=torch.float32, device=dev)
for name, shape, up, down, pad, gain in [
        ("down2 [64,128,128,128]", (64, 128, 128, 128), 1, 2, (1, 1), 1),
        ("up2 [64,256,64,64]", (64, 256, 64, 64), 2, 1, (2, 1), 4),
        ("down2 [64,256,64,64]", (64, 256, 64, 64), 1, 2, (1, 1), 1),
        ("fir [64,128,64,64] pad2", (64, 128, 64, 64), 1, 1, (2, 2), 1),
        ("down2 [64,256,32,32]", (64, 256, 32, 32), 1, 2, (1, 1), 1),
        ("up2 [64,256,16,16]", (64, 256, 16, 16), 2, 1, (2, 1), 4)]:
    x = torch.randn(shape, device=dev)
    y = upfirdn2d(x, k * gain, up=up, down=down, pad=pad)
    t = t_of(lambda: upfirdn2d(x, k * gain, up=up, down=down, pad=pad))
    gbs = 4 * (x.numel() + y.numel()) / t / 1e9
    res["upfirdn2d " + name] = {"ms": round(t * 1e3, 4), "GB/s": round(gbs, 1),
                                "hbm_frac": round(gbs / 8000, 3)}
for (N, C, H, G) in [(64, 128, 128, 32), (64, 256, 64, 32), (64, 384, 128, 32), (64, 256, 16, 32)]:
    x = torch.randn(N, C, H, H, device=dev)
    w = torch.randn(C, device=dev)
    b = torch.randn(C, device=dev)
    bnc = torch.randn(N, C, device=dev)
    with torch.no_grad():
        t = t_of(lambda: group_norm_act_f(x, G, w, b, 1e-6, 1, bnc))
    gbs = 8 * x.numel() / t / 1e9
    res[f"gn_silu [{N},{C},{H},{H}] G{G}"] = {"ms": round(t * 1e3, 4), "GB/s": round(gbs, 1),
                                              "hbm_frac": round(gbs / 8000, 3)}
x = torch.randn(64, 128, 128, 128, device=dev)
h = torch.randn_like(x)
bb = torch.randn(128, device=dev)
with torch.no_grad():
    t = t_of(lambda: residual_rescale(x, h, bb, 2 ** 0.5))
res["residual [64,128,128,128]"] = {"ms": round(t * 1e3, 4), "GB/s": round(12 * x.numel() / t / 1e9, 1)}
# ns_step: simulator shape (pinn_kalman/simulator.py:49-52): B=256, 192x192, dt=0.0025, dx=0.005
from op import ns_step
g = torch.Generator(device=dev).manual_seed(0)
B, n = 256, 192
f = torch.rand(B, 1, n, n, device=dev, generator=g) * 0.9 + 0.1
p = torch.randn(B, 1, n, n, device=dev, generator=g) * 0.01
v = (torch.rand(B, 2, n, n, device=dev, generator=g) * 0.45 + 0.05) * \
    torch.sign(torch.randn(B, 2, n, n, device=dev, generator=g))
sites = B * n * n
t = t_of(lambda: ns_step.full_step(f, v, p, 0.0025, 0.005))
res["ns_step full_step fused B256 192^2"] = {"ms": round(t * 1e3, 4),
                                            "Gsite/s": round(sites / t / 1e9, 2),
                                            "GB/s@32B/site": round(32 * sites / t / 1e9, 1)}
def three():
    v1 = ns_step.update_velocity(v, p, 0.0025, 0.005)
    p1 = ns_step.update_pressure(p, v1, 0.0025, 0.005)
    return ns_step.update_density(f, v1, 0.0025, 0.005)
t = t_of(three)
res["ns_step 3 reference ops B256 192^2"] = {"ms": round(t * 1e3, 4),
                                            "Gsite/s": round(sites / t / 1e9, 2),
                                            "GB/s@32B/site": round(32 * sites / t / 1e9, 1)}
print(json.dumps(res, indent=1))
