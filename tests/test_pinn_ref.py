"""CPU: pin the oracle's PINN restatement (oracle/pinn_ref.py, bench.py's PINN CPU baseline)
against the reference-generated fixtures -- pinn_fwd.npz (16^2, feature_nums [4, 8, 8]) and
cfg_pinn64.npz (configs[3] as shipped, 64^2) -- and its vectorised correlation against the
loop restatement oracle/correlation_ref.py.  Tolerances as the GPU tests: flows / pressure
1e-4 relative to max|ref|, equation_mse and its input sensitivities 2e-3."""
import numpy as np
import pytest
import torch

from conftest import build_pinn_weights, full_pinn_config, load_golden, small_config
from oracle import correlation_ref as cr
from oracle import pinn_ref


def _rel(a, ref):
    a, ref = np.asarray(a, np.float64), np.asarray(ref, np.float64)
    return float(np.abs(a - ref).max() / max(np.abs(ref).max(), 1e-30))


def test_vectorised_correlation_matches_loop_restatement():
    g = torch.Generator().manual_seed(0)
    a = torch.randn(2, 5, 9, 11, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.randn(2, 5, 9, 11, generator=g, dtype=torch.float64, requires_grad=True)
    out = pinn_ref.correlation(a, b)
    np.testing.assert_allclose(out.detach().numpy(), cr.forward(a.detach().numpy(), b.detach().numpy()),
                               rtol=1e-12, atol=1e-12)
    go = torch.randn(out.shape, generator=g, dtype=torch.float64)
    ga, gb = torch.autograd.grad(out, (a, b), go)
    ra, rb = cr.backward(a.detach().numpy(), b.detach().numpy(), go.numpy())
    np.testing.assert_allclose(ga.numpy(), ra, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(gb.numpy(), rb, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("fixture,cfg_fn", [("pinn_fwd.npz", small_config),
                                            ("cfg_pinn64.npz", full_pinn_config)])
def test_pinn_ref_matches_reference_fixture(fixture, cfg_fn):
    from configs.pinn import pinn_pde
    from pinn_kalman.pinn import PINN
    d = load_golden(fixture)
    c = cfg_fn(pinn_pde.get_config)
    P = pinn_ref.init_params(build_pinn_weights(PINN, c).state_dict())
    T = lambda k: torch.tensor(d[k])
    x, y, t = (T(k).requires_grad_() for k in ("x", "y", "t"))
    flows, pres = pinn_ref.forward(P, c, T("f1"), T("f2"), x, y, t)
    assert len(flows) == int(d["n_flows"])
    for i, fl in enumerate(flows):
        assert _rel(fl.detach(), d[f"flow{i}"]) <= 1e-4, f"flow{i}"
    assert _rel(pres.detach(), d["pres"]) <= 1e-4
    eq7 = pinn_ref.equation_mse(x, y, t, flows[-1], pres, 10000000.0)
    assert _rel(eq7.item(), d["eq7"]) <= 2e-3
    eq50 = pinn_ref.equation_mse(x, y, t, flows[-1], pres, 50.0)
    assert _rel(eq50.item(), d["eq50"]) <= 2e-3
    gx, gy, gt = torch.autograd.grad(eq50, (x, y, t), retain_graph=True)
    for nm, v in (("gx", gx), ("gy", gy), ("gt", gt)):
        assert _rel(v, d[nm]) <= 2e-3, nm
    eq50.backward()  # the double backward runs through grid_sample_ref.grad2
    assert all(torch.isfinite(p.grad).all() for p in P.values() if p.grad is not None)
