"""PINN graph bisect: capture part of the PINN step (DIAG9 = flow | pres | data | full |
fwd_full), replay, allocate-fill-free NaN poison, replay again: a part whose replay changes
after the poison reads memory it does not own.  B=64 bench batch, one fixed mask."""
import contextlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
from configs.pinn import pinn_pde  # noqa: E402
from pinn_kalman.pinn import PINN  # noqa: E402

MODE = os.environ.get("DIAG9", "full")
B = int(os.environ.get("DIAG_B", 64))
dev = torch.device("cuda:0")
if os.environ.get("DIAG_FREED") == "1":
    torch.cuda.memory._record_memory_history(max_entries=500000)
c = pinn_pde.get_config()
c.device = dev
torch.manual_seed(0)
model = PINN(c).train()
g = torch.Generator().manual_seed(3)
mask = (torch.rand(B, 1, 64, 64, generator=g) > 0.1).float().to(dev)
batch = bench.pinn_batch(c, B, dev, seed=0)
sb = tuple(t.detach().clone().requires_grad_(t.requires_grad) for t in batch)
params = [p for p in model.parameters() if p.requires_grad]


def loss_fn():
    f1, f2, x, y, t, target = sb
    f1, f2 = mask * f1, mask * f2
    if MODE == "flow":
        flow = model.flownet(f1, f2, x, y, t)
        l = model.flownet.multiscale_data_mse(flow, target)
        return l, l
    if MODE == "pres":
        with torch.no_grad():
            flow = model.flownet(f1, f2, x, y, t)
        flow = [f.detach() for f in flow]
        p = model.pressurenet(flow, x, y, t)
        l = model.pressurenet.data_mse(p, target)
        return l, l
    flow, pres = model(f1, f2, x, y, t)
    data = model.flownet.multiscale_data_mse(flow, target) + model.pressurenet.data_mse(pres, target)
    if MODE == "data":
        return data, data
    pinn = model.equation_mse(x, y, t, flow[-1], pres, 1e7) * c.training.pinn_loss_weight
    return pinn + data, pinn


bwd = MODE not in ("fwd_full", "eager_fwd_full")
EAGER = MODE.startswith("eager_")
MODE = MODE.replace("eager_", "").replace("fwd_full", "full")
if EAGER:  # no graph: the same part run eagerly, poison between two runs
    def run():
        global out
        for t in params + list(sb):
            t.grad = None
        o = loss_fn()
        if bwd:
            o[0].backward()
        out = tuple(v.detach() for v in o)

    class _G:
        replay = staticmethod(run)
    MODE = "eager " + MODE
WARM_SIDE = os.environ.get("DIAG_WARM", "cur") == "side"
side = torch.cuda.Stream(dev) if WARM_SIDE else torch.cuda.current_stream(dev)
side.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(side):
    for _ in range(2):
        out = loss_fn()
        if bwd:
            out[0].backward()
torch.cuda.current_stream(dev).wait_stream(side)
del out
for t in params + list(sb):
    t.grad = None
FREED = os.environ.get("DIAG_FREED") == "1"


def active_blocks():
    res = {}
    for seg in torch.cuda.memory._snapshot()["segments"]:
        a = seg["address"]
        for b in seg["blocks"]:
            if b["state"] == "active_allocated":
                res[a] = (b["size"], seg.get("segment_pool_id"), b.get("frames", []))
            a += b["size"]
    return res


if FREED:
    torch.cuda.synchronize()
    before = active_blocks()
graph = _G() if EAGER else torch.cuda.CUDAGraph(keep_graph=True)
with contextlib.nullcontext() if EAGER else torch.cuda.graph(graph):
    out = loss_fn()
    if bwd:
        out[0].backward()
out = tuple(o.detach() for o in out)
if not EAGER:
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from graph_topology import classify, copy_nodes, topology
    graph.instantiate()
    print("topology", topology(graph.raw_cuda_graph()), flush=True)
    segs = torch.cuda.memory._snapshot()["segments"]
    cps, n = copy_nodes(graph.raw_cuda_graph())
    import collections
    cnt = collections.Counter()
    for c_ in cps:
        if c_[1] == "memcpy":
            key = ("memcpy", c_[5], classify(c_[2], segs), classify(c_[3], segs))
        else:
            key = ("memset", classify(c_[2], segs))
        cnt[key] += 1
        if "not-torch" in key or any("(0, 0)" in str(k) for k in key):
            print("   outside the graph pool:", c_, key, flush=True)
    print("copy/memset nodes by (kind, src pool, dst pool):", dict(cnt), flush=True)
if FREED:
    import gc
    gc.collect()
    after = active_blocks()
    print(f"{len(before)} active blocks before capture, {len(after)} after", flush=True)
    for a, (sz, pool, fr) in sorted(before.items()):
        if a not in after:
            names = [f"{f['filename'].split('/')[-1]}:{f['line']}:{f['name']}" for f in fr
                     if f["filename"].endswith(".py")][:8]
            print(f"  freed: {hex(a)} size {sz} pool {pool} alloc at {names}", flush=True)


pnames = [n for n, p in model.named_parameters() if p.requires_grad]


def snap():
    return ([("out0", out[0].clone()), ("out1", out[1].clone())]
            + [(n, p.grad.clone()) for n, p in zip(pnames, params) if p.grad is not None])


def cmp(tag, a, b):
    rows = []
    for (n, x), (_, y) in zip(a, b):
        scale = float(y.abs().max()) + 1e-30
        d = float((x - y).abs().max()) / scale
        rows.append((d if d == d else float("inf"), n, scale, float(x.abs().max())))
    rows.sort(reverse=True)
    nf = sum(not bool(torch.isfinite(x).all()) for _, x in a)
    print(f"{MODE}{'' if bwd else ' (fwd only)'} {tag}: nonfinite {nf}",
          [float(x) for _, x in a[:2]], flush=True)
    for d, n, sc, mx in rows[:6]:
        print(f"    {n}: rel diff {d:.2e} (ref max {sc:.2e}, this max {mx:.2e})", flush=True)


def poison(total_mb=8192):
    held, n, sz = [], 0, 1 << 10
    while n < total_mb << 20:
        held.append(torch.full((sz // 4,), float("nan"), device=dev))
        n += sz
        sz = sz * 2 if sz < (64 << 20) else (1 << 10)
    torch.cuda.synchronize()
    del held


graph.replay()
torch.cuda.synchronize()
s1 = snap()
graph.replay()
torch.cuda.synchronize()
cmp("replay2 vs 1", snap(), s1)
poison()
graph.replay()
torch.cuda.synchronize()
cmp("after poison vs 1", snap(), s1)
