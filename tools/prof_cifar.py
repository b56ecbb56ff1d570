"""configs[1] CIFAR-10 NCSN++ train steps (B=128) for rocprofv3: bench.bench_cifar_train's
warm-up + 3 timed steps."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import dist  # noqa: E402

sys.argv = ["bench.py", "--cifar-steps", "3"]
args = bench.parse()
ctx = dist.init_from_env()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
print(bench.bench_cifar_train(args, ctx, dev), flush=True)
