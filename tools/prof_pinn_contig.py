"""Which call sites of the PINN train step (configs[3], B=64) make .contiguous() copy, and the
tensor strides they get (one step after warm-up; Python-level attribution)."""
import os, sys, collections, traceback
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
import bench
from dist import DistContext
class A: pass
args = A(); args.batch = 64; args.pinn_warmup = 3; args.pinn_steps = 1; args.pinn_graph = False
dev = torch.device("cuda:0")
bench.bench_pinn(args, DistContext(), dev)
sites = collections.Counter()
orig = torch.Tensor.contiguous
def contig(self, *a, **k):
    if not self.is_contiguous(*a, **k):
        fr = [f for f in traceback.extract_stack()[:-1] if "b-pinn-kalman-filter_amd" in f.filename]
        where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[::-1][:4])
        kind = "expanded" if 0 in self.stride() else "strided"
        sites[(where, kind)] += 1
    return orig(self, *a, **k)
torch.Tensor.contiguous = contig
args.pinn_warmup = 0
bench.bench_pinn(args, DistContext(), dev)
print("copies", sum(sites.values()))
for (w, kind), n in sites.most_common(40):
    print(f"{n:5d} {kind:8s} {w}")
