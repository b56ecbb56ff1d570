"""One implicit-GEMM conv call repeated (for rocprofv3 --pmc passes and quick timing):
python tools/igemm_one.py MODE N C H W Cout K STRIDE PAD [REPS]   (MODE fwd | dgrad | wgrad)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

from op import conv as C  # noqa: E402

mode = sys.argv[1]
N, Ci, H, W, Co, K, s, p = (int(v) for v in sys.argv[2:10])
reps = int(sys.argv[10]) if len(sys.argv) > 10 else 20
dev = torch.device("cuda:0")
x = torch.randn(N, Ci, H, W, device=dev)
w = torch.randn(Co, Ci, K, K, device=dev) * 0.05
Ho, Wo = (H + 2 * p - K) // s + 1, (W + 2 * p - K) // s + 1
gy = torch.randn(N, Co, Ho, Wo, device=dev)
fn = {"fwd": lambda: C.conv2d_igemm_raw(x, w, None, s, p),
      "dgrad": lambda: C.conv2d_input_igemm_raw(x.shape, w, gy, s, p),
      "wgrad": lambda: C.conv2d_weight_igemm_raw(x, w.shape, gy, s, p, False)}[mode]
for _ in range(3):
    fn()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    fn()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / reps * 1e3
fl = 2.0 * N * Ci * Co * K * K * Ho * Wo
print(f"{mode} N={N} {Ci}->{Co} {H}x{W} k{K} s{s} p{p}: {us:.1f} us, {fl / us / 1e6:.1f} TFLOP/s", flush=True)
