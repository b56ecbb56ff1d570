"""Host-side profile of the PINN train step (cProfile over 3 steps after 2 warm-up steps):
where the CPU time of the launch-bound step goes."""
import cProfile, os, pstats, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
import bench
from dist import DistContext

class A: pass
args = A(); args.batch = 64; args.pinn_warmup = 2; args.pinn_steps = 2; args.pinn_graph = False
dev = torch.device("cuda:0")
bench.bench_pinn(args, DistContext(), dev)  # warm-up incl. MIOpen finds
pr = cProfile.Profile()
args.pinn_warmup = 0; args.pinn_steps = 3
pr.enable()
print(bench.bench_pinn(args, DistContext(), dev), flush=True)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(45)
st.sort_stats("cumulative").print_stats(40)
