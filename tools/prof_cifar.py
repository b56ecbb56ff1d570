"""configs[1] CIFAR-10 NCSN++ train steps for rocprofv3: 2 warm-up + 3 steps."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
import bench
from dist import DistContext
class A: pass
args = A(); args.cifar_steps = 3
print(bench.bench_cifar_train(args, DistContext(), torch.device("cuda:0")), flush=True)
