"""Quick GPU probe: loads libbpk.so next to torch's HIP runtime, checks a few
kernels against torch CPU math, times MIOpen fp32 convs of the NCSN++ shapes."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "b-pinn-kalman-filter_amd"))
import torch
import torch.nn.functional as F
print("torch", torch.__version__, "hip", torch.version.hip, "dev", torch.cuda.get_device_name(0))
from op import upfirdn2d, norm_act
from op import _lib
print("abi", _lib.lib.bpk_abi_version())
dev = "cuda"
torch.manual_seed(0)
# upfirdn2d vs a direct CPU restatement
def ref_upfirdn(x, k, up, down, pad):
    N, C, H, W = x.shape
    kh, kw = k.shape
    U = torch.zeros(N, C, H * up, W * up, dtype=x.dtype)
    U[:, :, ::up, ::up] = x
    P = F.pad(U, (pad[0], pad[1], pad[0], pad[1]))
    out = F.conv2d(P.reshape(N * C, 1, *P.shape[2:]), torch.flip(k, [0, 1])[None, None])
    out = out[:, :, ::down, ::down]
    return out.reshape(N, C, *out.shape[2:])
k = torch.tensor([1., 3, 3, 1]); k = torch.outer(k, k); k = k / k.sum()
for (up, down, pad, kk) in [(1, 2, (1, 1), k), (2, 1, (2, 1), k * 4), (1, 1, (2, 2), k)]:
    x = torch.randn(2, 3, 32, 32)
    y = upfirdn2d(x.to(dev), kk.to(dev), up=up, down=down, pad=pad).cpu()
    r = ref_upfirdn(x, kk, up, down, pad)
    print("upfirdn", up, down, pad, tuple(y.shape), "maxerr", (y - r).abs().max().item())
# group norm + silu
gn = torch.nn.GroupNorm(8, 32, eps=1e-6)
x = torch.randn(4, 32, 16, 16)
y = norm_act.group_norm_act(x.to(dev), gn.to(dev)).cpu()
r = F.silu(gn.cpu()(x))
print("gn_silu maxerr", (y - r).abs().max().item())
# conv timing (MIOpen fp32)
torch.backends.cudnn.benchmark = True
for (B, Ci, Co, H) in [(64, 128, 128, 128), (64, 256, 256, 64), (64, 256, 256, 32), (64, 512, 256, 64)]:
    x = torch.randn(B, Ci, H, H, device=dev)
    w = torch.randn(Co, Ci, 3, 3, device=dev) * 0.01
    for _ in range(3): F.conv2d(x, w, padding=1)
    torch.cuda.synchronize()
    t0 = time.time(); n = 10
    for _ in range(n): F.conv2d(x, w, padding=1)
    torch.cuda.synchronize(); dt = (time.time() - t0) / n
    fl = 2 * B * Co * Ci * 9 * H * H
    print(f"conv3x3 B{B} {Ci}->{Co} @{H}: {dt*1e3:.2f} ms  {fl/dt/1e12:.1f} TF/s (fp32)")
    xb, wb = x.bfloat16(), w.bfloat16()
    for _ in range(3): F.conv2d(xb, wb, padding=1)
    torch.cuda.synchronize(); t0 = time.time()
    for _ in range(n): F.conv2d(xb, wb, padding=1)
    torch.cuda.synchronize(); dt = (time.time() - t0) / n
    print(f"   bf16: {dt*1e3:.2f} ms  {fl/dt/1e12:.1f} TF/s")
    xc = x.to(memory_format=torch.channels_last)
    for _ in range(3): F.conv2d(xc, w.to(memory_format=torch.channels_last), padding=1)
    torch.cuda.synchronize(); t0 = time.time()
    for _ in range(n): F.conv2d(xc, w.to(memory_format=torch.channels_last), padding=1)
    torch.cuda.synchronize(); dt = (time.time() - t0) / n
    print(f"   fp32 NHWC: {dt*1e3:.2f} ms  {fl/dt/1e12:.1f} TF/s")
print("PROBE OK")
