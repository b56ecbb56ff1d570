"""The NCSN++ 128^2 FIR-down convs (conv_downsample_2d: upfirdn2d pad(2,2) then a 3x3 stride-2
conv, reference up_or_down_sampling.py:144-178, layerspp.py:149-163): implicit-GEMM kernel vs
MIOpen per shape, HIP-event timed (20 reps), at the bench batch (64) and the per-rank batch
of the 8-GPU point (8)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from op import conv as C  # noqa: E402

dev = torch.device("cuda:0")


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for B in (64, 8):
    for cin, cout, hin in ((1, 128, 129), (128, 256, 65), (256, 256, 33)):
        x = torch.randn(B, cin, hin, hin, device=dev)
        w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
        b = torch.randn(cout, device=dev)
        ho = (hin - 3) // 2 + 1
        fl = 2.0 * B * cin * cout * 9 * ho * ho
        ti = timeit(lambda: C.conv2d_igemm_raw(x, w, b, (2, 2), (0, 0)))
        tm = timeit(lambda: F.conv2d(x, w, b, stride=2))
        err = (C.conv2d_igemm_raw(x, w, b, (2, 2), (0, 0)) - F.conv2d(x, w, b, stride=2)).abs().max().item()
        print(f"B={B:3d} {cin:3d}->{cout:3d} @{hin}: igemm {ti:8.1f} us ({fl / ti / 1e6:6.1f} TF/s)  "
              f"miopen {tm:8.1f} us ({fl / tm / 1e6:6.1f} TF/s)  maxdiff {err:.2e}", flush=True)
