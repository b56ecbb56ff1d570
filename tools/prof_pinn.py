"""PINN train steps (configs[3], B=64, 64x64) for rocprofv3: 2 warm-up + 3 profiled steps."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
import bench
from dist import DistContext

class A: pass
args = A(); args.batch = 64; args.pinn_warmup = 2; args.pinn_steps = 3; args.pinn_graph = False
dev = torch.device("cuda:0")
print(bench.bench_pinn(args, DistContext(), dev), flush=True)
