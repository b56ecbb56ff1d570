"""PINN train step under torch.profiler: aten conv ops grouped by input shapes (GPU time)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
import bench
from dist import DistContext
class A: pass
args = A(); args.batch = 64; args.pinn_warmup = 3; args.pinn_steps = 1; args.pinn_graph = False
dev = torch.device("cuda:0")
bench.bench_pinn(args, DistContext(), dev)
from torch.profiler import profile, ProfilerActivity
args.pinn_warmup = 0; args.pinn_steps = 1
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    bench.bench_pinn(args, DistContext(), dev)
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=45, max_name_column_width=40, max_shapes_column_width=90))
