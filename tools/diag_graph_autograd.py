"""Minimal pure-aten repro: nn.Conv2d(3, 6, 3) -> x - mean_hw(x), backward captured in a
hipGraph; compares the bias gradient of replays 0..2 with eager under capture variants
(V = warm-up on a side stream / none / on the current stream; relaxed capture mode)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from graph_topology import classify, copy_nodes, topology  # noqa: E402

dev = torch.device("cuda:0")


class Sub(torch.nn.Module):
    def forward(self, x):
        return x - x.mean(dim=(2, 3), keepdim=True)


class Affine(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.randn(6, 3))
        self.bias = torch.nn.Parameter(torch.randn(6))

    def forward(self, x):
        return torch.einsum("oc,nchw->nohw", self.weight, x) + self.bias[None, :, None, None]


def make(conv):
    if conv == "miopen":
        return torch.nn.Conv2d(3, 6, 3, padding=1)
    if conv == "native":
        from models import layers
        return layers.Conv2d(3, 6, 3, padding=1)
    return Affine()


def case(variant, root="clone", conv="miopen"):
    torch.manual_seed(0)
    mod = torch.nn.Sequential(make(conv), Sub()).to(dev)
    params = list(mod.parameters())
    x = torch.randn(64, 3, 64, 64, device=dev, requires_grad=True)
    gy = torch.randn(64, 6, 64, 64, device=dev)

    def step():
        mod(x).backward(gy.clone() if root == "clone" else gy * 1.0)

    step()
    ref = [p.grad.clone() for p in params]
    if variant == "side":
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
            step()
        torch.cuda.current_stream().wait_stream(s)
    elif variant == "cur":
        step()
    for p in params + [x]:
        p.grad = None
    g = torch.cuda.CUDAGraph(keep_graph=True)
    kw = {"capture_error_mode": "relaxed"} if variant == "relaxed" else {}
    with torch.cuda.graph(g, **kw):
        step()
    g.instantiate()
    print(variant, conv, topology(g.raw_cuda_graph()), flush=True)
    segs = torch.cuda.memory._snapshot()["segments"]
    cps, n = copy_nodes(g.raw_cuda_graph())
    for c in cps:
        if c[1] == "memcpy":
            print(f"   node {c[0]}/{n} memcpy {c[4]} B kind {c[5]} src {hex(c[2])} "
                  f"({classify(c[2], segs)}) dst {hex(c[3])} ({classify(c[3], segs)})")
        else:
            print(f"   node {c[0]}/{n} memset {c[3]} B value {c[4]} dst {hex(c[2])} "
                  f"({classify(c[2], segs)})")
    print("   gy", hex(gy.data_ptr()), "x", hex(x.data_ptr()), "grads",
          [hex(p.grad.data_ptr()) for p in params], flush=True)
    out = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        out.append(float((params[1].grad - ref[1]).abs().max()))
    print(f"{variant} conv={conv}: |bias grad - eager| per replay {['%.2e' % v for v in out]} "
          f"(eager |bias grad| max {float(ref[1].abs().max()):.2e})", flush=True)


sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             "b-pinn-kalman-filter_amd")]
for v in ("side", "cur"):
    for cv in ("miopen", "native", "affine"):
        case(v, conv=cv)


