"""PINN train step (configs[3], B=64) under torch.profiler with Python stacks: for the aten
ops issued most often (copies, sums, fills, elementwise), the call sites that issue them."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import collections
import torch
import bench
from dist import DistContext
from torch.profiler import profile, ProfilerActivity
class A: pass
args = A(); args.batch = 64; args.pinn_warmup = 3; args.pinn_steps = 1; args.pinn_graph = False
dev = torch.device("cuda:0")
bench.bench_pinn(args, DistContext(), dev)
args.pinn_warmup = 0
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    bench.bench_pinn(args, DistContext(), dev)
want = ("aten::to", "aten::copy_", "aten::sum", "aten::fill_", "aten::mul", "aten::add_",
        "aten::add", "aten::zeros_like", "aten::clone", "aten::contiguous", "aten::div")
agg = collections.defaultdict(collections.Counter)
evs = prof.events()
names = collections.Counter(ev.name for ev in evs)
print("events", len(evs), "with stack", sum(1 for ev in evs if ev.stack), names.most_common(12))
shown = 0
for ev in evs:
    if ev.name in want and shown < 3:
        print("sample", ev.name, ev.thread, list(ev.stack)[:6])
        shown += 1
for ev in evs:
    if ev.name in want:
        frames = [f for f in (ev.stack or []) if ".py" in f and "profiler" not in f]
        site = " <- ".join(f.split("/")[-1] for f in frames[:4]) if frames else f"<no python stack, thread {ev.thread}>"
        agg[ev.name][site] += 1
for name in want:
    c = agg[name]
    print(f"== {name}: {sum(c.values())}")
    for site, n in c.most_common(8):
        print(f"  {n:5d}  {site[:230]}")
