"""Launch drivers for the round-2 rocprofv3 --pmc passes (one counter group per pass):
   wino_one  one PRE+stats Winograd launch 128->128 @128^2 at B=16 after 2 warm-ups
             (a single dispatch small enough that SQ_VALU_MFMA_BUSY_CYCLES does not saturate)
   mix       the NCSN++ PRE-conv mix of bench.conv_roofline, once (B = 64)
   ns        3 ns_step full steps, B = 256 x 192^2
   upfirdn   the four bench upfirdn2d shapes, 3 launches each (B = 64)
   wgrad_one the Winograd weight gradient 128->128 @128^2 at B=16, 3 launches
   igemm_set the PINN step's heaviest implicit-GEMM shapes (B = 64), 3 launches each:
             fwd 34->128 @32^2, dgrad 128->49 and 128->34 @32^2, wgrad 128->16 @64^2 (bias)
Kernel names / grid sizes in the counter CSV identify the dispatches."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
mode = sys.argv[1]
g = torch.Generator(device=dev).manual_seed(0)
if mode in ("wino_one", "mix"):
    from op.conv import conv3x3, filter_transform
    rows = [(128, 128, 128, 1, 0)] if mode == "wino_one" else bench.WINO_MIX
    B = 16 if mode == "wino_one" else 64
    for cin, cout, hw, n_pre, n_res in rows:
        x = torch.randn(B, cin, hw, hw, device=dev, generator=g)
        w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) / (3 * cin ** 0.5)
        b = torch.randn(cout, device=dev, generator=g)
        pre = torch.stack([torch.rand(B, cin, device=dev, generator=g) + 0.5,
                           torch.randn(B, cin, device=dev, generator=g) * 0.1], -1).contiguous()
        skip = torch.randn(B, cout, hw, hw, device=dev, generator=g)
        filter_transform(w)
        if mode == "wino_one":
            for _ in range(3):
                conv3x3(x, w, b, pre=pre, stats=True)
        else:
            for _ in range(n_pre):
                conv3x3(x, w, b, pre=pre, stats=True)
            for _ in range(n_res):
                conv3x3(x, w, b, skip=skip, div=2 ** 0.5, pre=pre, stats=True)
        torch.cuda.synchronize()
        del x, skip
elif mode == "wgrad_one":
    from op.conv import conv3x3_wgrad_raw
    x = torch.randn(16, 128, 128, 128, device=dev, generator=g)
    gy = torch.randn(16, 128, 128, 128, device=dev, generator=g)
    for _ in range(3):
        conv3x3_wgrad_raw(x, gy, (128, 128, 3, 3))
elif mode == "igemm_set":
    from op.conv import conv2d_igemm_raw, conv2d_input_igemm_raw, conv2d_weight_igemm_raw
    x = torch.randn(64, 34, 32, 32, device=dev, generator=g)
    w = torch.randn(128, 34, 3, 3, device=dev, generator=g)
    for _ in range(3):
        conv2d_igemm_raw(x, w, None, 1, 1)
    gy = torch.randn(64, 128, 32, 32, device=dev, generator=g)
    for c in (49, 34):
        w = torch.randn(128, c, 3, 3, device=dev, generator=g)
        for _ in range(3):
            conv2d_input_igemm_raw((64, c, 32, 32), w, gy, 1, 1)
    x = torch.randn(64, 128, 64, 64, device=dev, generator=g)
    gy = torch.randn(64, 16, 64, 64, device=dev, generator=g)
    for _ in range(3):
        conv2d_weight_igemm_raw(x, (16, 128, 3, 3), gy, 1, 1, True)
elif mode == "ns":
    from op import ns_step
    f, v, p = (torch.tensor(a, device=dev) for a in bench._ns_fields(np.random.default_rng(0), 256, 192))
    for _ in range(3):
        f, v, p = ns_step.full_step(f, v, p, 0.0025, 0.005)
elif mode == "upfirdn":
    from op import upfirdn2d
    k = torch.tensor(np.outer([1, 3, 3, 1], [1, 3, 3, 1]) / 64.0, dtype=torch.float32, device=dev)
    for name, (c, hw), kw, gain in bench.UPFIRDN_SHAPES:
        x = torch.randn(64, c, hw, hw, device=dev, generator=g)
        for _ in range(3):
            upfirdn2d(x, k * gain, **kw)
        torch.cuda.synchronize()
        del x
torch.cuda.synchronize()
print("ok", mode)
