"""Per-parameter error report of the PINN fixtures on the GPU (diagnostic)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO, os.path.join(REPO, "tests"),
                os.path.join(REPO, "tests", "golden")]
import numpy as np, torch
from conftest import load_golden
from make_golden_pinn import sample_idx
import test_gpu_pinn as T

dev = torch.device("cuda:0")
d = load_golden("pinn_fwd.npz")
c, m = T._model(dev)
m.train()
G = lambda k: torch.tensor(d[k], device=dev)
x, y, t = (G(k).requires_grad_() for k in ("x", "y", "t"))
mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
for rep in range(2):
    m.zero_grad()
    flows, pres = m(G("f1"), G("f2"), x, y, t)
    if mode == "full":
        eq7 = m.equation_mse(x, y, t, flows[-1], pres, 10000000.0)
        m.zero_grad()
    eq50 = m.equation_mse(x, y, t, flows[-1], pres, 50.0)
    if mode == "full":
        torch.autograd.grad(eq50, (x, y, t), retain_graph=True)
    eq50.backward()
    print("mode", mode, "rep", rep)
    for k, p in m.named_parameters():
        if "g:" + k in d.files:
            v = p.grad.reshape(-1).cpu().numpy()[sample_idx(p.numel())]
            r = d["g:" + k]
            if np.abs(v - r).max() > 0.005 * max(np.abs(r).max(), 1e-5):
                print(f"{k:60s} max|ref| {np.abs(r).max():.3e} max|diff| {np.abs(v - r).max():.3e}")
