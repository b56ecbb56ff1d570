"""upfirdn2d on the four SURVEY 8(d) shapes (B = 64): HIP-event time per launch over graph
replays of 20 launches (bench.time_kernel_graph; the scaled FIR taps prepared outside) and the fraction of the
8 TB/s HBM peak on the algorithmic bytes 4 (in + out).  Env switches of csrc/upfirdn2d.hip
select variants for A/B runs."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from op import upfirdn2d  # noqa: E402

dev = torch.device("cuda:0")
k = torch.tensor(np.outer([1, 3, 3, 1], [1, 3, 3, 1]) / 64.0, dtype=torch.float32, device=dev)
st = torch.cuda.Stream(dev)
tag = os.environ.get("TAG", "")
for name, (c, hw), kw, gain in bench.UPFIRDN_SHAPES:
    x = torch.randn(64, c, hw, hw, device=dev)
    kg = (k * gain).contiguous()
    t = bench.time_kernel_graph(lambda: upfirdn2d(x, kg, **kw), st, reps=20)
    ho = bench._upfirdn_out(hw, kw)
    nbytes = 4.0 * (x.numel() + 64 * c * ho * ho)
    print(f"{tag} {name}: {t * 1e6:7.1f} us  {nbytes / t / 1e9:7.0f} GB/s  frac {nbytes / t / 8e12:.3f}",
          flush=True)
