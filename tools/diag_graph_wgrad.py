"""The Winograd weight + bias gradient alone (conv3x3_wgrad_raw, bias_grad=True) captured in a
hipGraph and replayed with NaN poison / eager work in between; also the whole _Conv3x3
forward + backward (autograd) of one 64->64 conv."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

from op import conv  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)


def poison(mb=2048):
    held, n, sz = [], 0, 1 << 9
    while n < mb << 20:
        held.append(torch.full((max(sz // 4, 1),), float("nan"), device=dev))
        n += sz
        sz = sz * 2 if sz < (64 << 20) else (1 << 9)
    torch.cuda.synchronize()


def run(name, body, outs_fn, ref):
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    res = []
    for k in range(4):
        if k >= 2:
            poison()
        g.replay()
        torch.cuda.synchronize()
        res.append(["%.1e" % (float((a - b).abs().max()) / (float(b.abs().max()) + 1e-30))
                    for a, b in zip(outs_fn(), ref)])
    print(name, "rel err per replay (replays 2, 3 after poison):", res, flush=True)


for (N, C, Co, H) in ((64, 64, 64, 64), (64, 32, 64, 64), (64, 64, 128, 32)):
    x = torch.randn(N, C, H, H, device=dev)
    gy = torch.randn(N, Co, H, H, device=dev)
    dw0, db0 = conv.conv3x3_wgrad_raw(x, gy, (Co, C, 3, 3), bias_grad=True)
    st = {}

    def body():
        st["dw"], st["db"] = conv.conv3x3_wgrad_raw(x, gy, (Co, C, 3, 3), bias_grad=True)
    run(f"wgrad+bias {N},{C}->{Co}@{H}", body, lambda: (st["dw"], st["db"]), (dw0.clone(), db0.clone()))

    w = (torch.randn(Co, C, 3, 3, device=dev) * 0.05).requires_grad_(True)
    b = torch.zeros(Co, device=dev, requires_grad=True)
    xr = x.clone().requires_grad_(True)
    y = conv.conv3x3(xr, w, b)
    y.backward(gy)
    ref = (w.grad.clone(), b.grad.clone(), xr.grad.clone())
    del y  # no AccumulateGrad node of this eager graph may survive into the capture

    def body2():
        conv.conv3x3(xr, w, b).backward(gy.clone())
    for t in (w, b, xr):
        t.grad = None
    body2()
    for t in (w, b, xr):
        t.grad = None
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body2()
    res = []
    for k in range(4):
        if k >= 2:
            poison()
        g.replay()
        torch.cuda.synchronize()
        res.append(["%.1e" % (float((t.grad - r).abs().max()) / (float(r.abs().max()) + 1e-30))
                    for t, r in zip((w, b, xr), ref)])
    print(f"autograd conv3x3 {N},{C}->{Co}@{H} (dw, db, dx)", res, flush=True)
