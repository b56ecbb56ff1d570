"""PINN residual sensitivities vs the float64 truth (tests/golden/*_f64.npz): prints the
error of gx/gy/gt and the worst parameter gradients, for A/B of conv / grid_sample paths
via env switches.  Usage: python tools/diag_pinn_f64.py [small|full]"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.environ.get("DIAG_PKG", os.path.join(REPO, "b-pinn-kalman-filter_amd"))
for p in (os.path.join(REPO, "tests"), REPO, PKG):
    sys.path.insert(0, p)
from conftest import (build_pinn_weights, full_pinn_config, load_golden, sample_idx,  # noqa
                      small_config)


def _swap_oracles():
    """DIAG_GS=oracle / DIAG_CORR=oracle: the fixture generator's stand-ins in the product
    model (ATen fwd/bwd + the torch grad2 restatement; numpy correlation)."""
    import types
    from models import flownet
    from oracle import correlation_ref as cr
    from oracle import grid_sample_ref as gsr
    if os.environ.get("DIAG_GS") == "oracle":
        class Bwd(torch.autograd.Function):
            @staticmethod
            def forward(ctx, go, inp, grid, pm, ac):
                ctx.save_for_backward(go, inp, grid)
                ctx.pm, ctx.ac = pm, ac
                return gsr.bwd(go, inp, grid, pm, ac)

            @staticmethod
            def backward(ctx, g2i, g2g):
                go, inp, grid = ctx.saved_tensors
                g2i = torch.zeros_like(inp) if g2i is None else g2i
                g2g = torch.zeros_like(grid) if g2g is None else g2g
                with torch.no_grad():
                    return (*gsr.grad2(g2i, g2g, go, inp, grid, ctx.pm, ctx.ac), None, None)

        class Fwd(torch.autograd.Function):
            @staticmethod
            def forward(ctx, inp, grid, pm, ac):
                ctx.save_for_backward(inp, grid)
                ctx.pm, ctx.ac = pm, ac
                return gsr.fwd(inp, grid, pm, ac)

            @staticmethod
            def backward(ctx, go):
                inp, grid = ctx.saved_tensors
                return (*Bwd.apply(go, inp, grid, ctx.pm, ctx.ac), None, None)

        flownet.grid_sample = types.SimpleNamespace(
            grid_sample_2d=lambda input, grid, padding_mode="zeros", align_corners=True:
            Fwd.apply(input, grid, ["zeros", "border"].index(padding_mode), align_corners))
    if os.environ.get("DIAG_CORR") == "oracle":
        class Corr(torch.autograd.Function):
            @staticmethod
            def forward(ctx, a, b, s):
                ctx.save_for_backward(a, b)
                ctx.s = s
                return torch.from_numpy(cr.forward(a.detach().cpu().numpy(), b.detach().cpu().numpy(), s)).to(a.device)

            @staticmethod
            def backward(ctx, g):
                a, b = ctx.saved_tensors
                gf, gs = cr.backward(a.detach().cpu().numpy(), b.detach().cpu().numpy(), g.detach().cpu().numpy(), ctx.s)
                return torch.from_numpy(gf).to(a.device), torch.from_numpy(gs).to(a.device), None

        flownet.correlation = types.SimpleNamespace(
            FunctionCorrelation=lambda a, b, stride: Corr.apply(a, b, stride))


def run(which):
    _swap_oracles()
    from configs.pinn import pinn_pde
    from pinn_kalman.pinn import PINN
    dev = torch.device("cuda:0")
    if which == "small":
        c, d, t = small_config(pinn_pde.get_config), load_golden("pinn_fwd.npz"), load_golden("pinn_fwd_f64.npz")
    else:
        c, d, t = full_pinn_config(pinn_pde.get_config), load_golden("cfg_pinn64.npz"), load_golden("cfg_pinn64_f64.npz")
    m = build_pinn_weights(PINN, c).to(dev)
    c.device = dev
    m.train()
    T = lambda k: torch.tensor(d[k], device=dev)
    x, y, tt = (T(k).requires_grad_() for k in ("x", "y", "t"))
    flows, pres = m(T("f1"), T("f2"), x, y, tt)
    if os.environ.get("DIAG_EQ7") == "1":
        eq7 = m.equation_mse(x, y, tt, flows[-1], pres, 10000000.0)
        out_eq7 = float(eq7)
    m.zero_grad()
    eq50 = m.equation_mse(x, y, tt, flows[-1], pres, 50.0)
    gx, gy, gt = torch.autograd.grad(eq50, (x, y, tt), retain_graph=True)
    eq50.backward()
    gscale = max(np.abs(t[k]).max() for k in t.files if k.startswith("g:"))
    out = {"which": which, "pkg": PKG, "env": {k: v for k, v in os.environ.items() if k.startswith("BPK_")}}
    for nm, v in (("gx", gx), ("gy", gy), ("gt", gt)):
        r = t[nm]
        out[nm] = [float(np.abs(v.cpu().numpy() - r).max() / np.abs(r).max()),
                   float(np.abs(d[nm] - r).max() / np.abs(r).max())]
    errs = []
    for k, p in m.named_parameters():
        if "g:" + k in t.files:
            r = t["g:" + k]
            v = p.grad.reshape(-1).cpu().numpy()[sample_idx(p.numel())]
            fl = max(np.abs(r).max(), 1e-4 * gscale)
            errs.append((float(np.abs(v - r).max() / fl), float(np.abs(d["g:" + k] - r).max() / fl), k,
                         v[:3].tolist(), r[:3].tolist()))
    errs.sort()
    out["worst_param"] = errs[-2:]
    out["fe02"] = [e for e in errs if e[2] == "flownet.feature_extractor.feature_extractors.0.2.bias"]
    out["eq7first"] = os.environ.get("DIAG_EQ7")
    out["swap"] = [os.environ.get("DIAG_GS"), os.environ.get("DIAG_CORR")]
    out["n_bad"] = sum(e[0] > 5e-3 for e in errs)
    out["bad_names"] = [e[2] for e in errs if e[0] > 5e-3][:40]
    print(json.dumps(out))


if __name__ == "__main__":
    run(sys.argv[1] if len(sys.argv) > 1 else "small")
