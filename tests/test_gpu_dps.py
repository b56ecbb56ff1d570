"""GPU parity of the DPS inverse sampler (device RK45 + HIP score net + input gradient)
against the reference-generated fixture tests/golden/dps.npz.

Tolerances: the drift probes 1e-4 relative to max|ref| (fp32 score net, its input
gradient and the DPS residual norm, same formulas, different summation order); the short
RK45 solve must accept the same time grid (1e-9 absolute on t) with the same number of
function evaluations, and reach the same state to 1e-4 relative."""
import numpy as np
import pytest
import torch

from conftest import load_golden, net_fixture, product_config

pytestmark = pytest.mark.gpu


def _setup(hip):
    import models  # noqa: F401
    import sde_lib
    from configs._configdict import ConfigDict
    from inverse.conditional_sampling import get_dps_sampler
    from inverse.operators import InpaintOperator
    from models import utils as mutils
    d = load_golden("dps.npz")
    cfg, sd, *_ = net_fixture("ddpm_a")
    c = product_config(cfg, hip)
    c.inverse = ConfigDict(dict(operator="inpaint", invert=False, ratio=0.5, sampler="dps",
                                variance=float(d["variance"]), solver="RK45"))
    model = mutils.create_model(c, wrap=False)
    model.load_state_dict({k: torch.tensor(v) for k, v in sd.items()}, strict=True)
    model.eval()
    mask = torch.tensor(d["mask"], device=hip)
    op = InpaintOperator(mask=[mask])
    y0 = op(torch.tensor(d["origin"], device=hip), keep_shape=False)
    sde = sde_lib.VPSDE(c.model.beta_min, c.model.beta_max, c.model.num_scales)
    obs = sde_lib.LOBSVSDE(sde, y0, op)
    shape = tuple(d["prior"].shape)
    noise = torch.tensor(d["obs_noise"], device=hip)
    sampler = get_dps_sampler(c, obs, shape, eps=float(d["eps"]), noise=noise)
    return d, model, sampler


def test_dps_drift_matches_reference(hip):
    d, model, sampler = _setup(hip)
    f = sampler.make_ode_func(model)
    x = torch.tensor(d["prior"], device=hip).reshape(-1).to(torch.float64)
    for tp, ref in zip(d["t_probe"], d["probes"]):
        out = f(float(tp), x).reshape(-1).double().cpu().numpy()
        err = np.abs(out - ref).max() / np.abs(ref).max()
        assert err < 1e-4, f"t={tp}: rel err {err:.2e}"


def test_dps_short_solve_matches_reference(hip):
    from inverse.conditional_sampling import get_solver
    d, model, sampler = _setup(hip)
    out = sampler(model, z=torch.tensor(d["prior"], device=hip))
    assert get_solver.last_nfe == int(d["nfe"])
    ref = d["sample"]
    err = np.abs(out.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err < 1e-4, f"rel err {err:.2e}"
