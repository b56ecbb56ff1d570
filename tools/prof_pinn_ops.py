"""PINN train step (configs[3], B=64) under torch.profiler: aten ops by call count and by
device time (which ops issue the step's ~13k launches)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
import bench
from dist import DistContext
from torch.profiler import profile, ProfilerActivity
class A: pass
args = A(); args.batch = 64; args.pinn_warmup = 3; args.pinn_steps = 1; args.pinn_graph = False
dev = torch.device("cuda:0")
bench.bench_pinn(args, DistContext(), dev)
args.pinn_warmup = 0
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    bench.bench_pinn(args, DistContext(), dev)
ka = prof.key_averages()
print(ka.table(sort_by="count", row_limit=40, max_name_column_width=50))
print(ka.table(sort_by="self_cuda_time_total", row_limit=30, max_name_column_width=50))
