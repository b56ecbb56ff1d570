"""PINN step time with MIOpen immediate mode vs exhaustive find (cudnn.benchmark)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
import bench
from dist import DistContext
torch.backends.cudnn.benchmark = bool(int(sys.argv[1]))
class A: pass
args = A(); args.batch = 64; args.pinn_warmup = 2; args.pinn_steps = 5; args.pinn_graph = False
t0 = time.time()
r = bench.bench_pinn(args, DistContext(), torch.device("cuda:0"))
print(sys.argv[1], round(time.time() - t0, 1), "s total", r["pinn_ms_per_step"], "ms/step", flush=True)
