"""Log-likelihood (bits/dim) through the probability-flow ODE (reference likelihood.py:24-113).

`get_likelihood_fn(sde, inverse_scaler, hutchinson_type, rtol, atol, method, eps)` ->
`likelihood_fn(model, data) -> (bpd, z, nfe)`.  The divergence is the Hutchinson-Skilling
estimate (one input-gradient of <drift, eps> per evaluation).  The augmented state
[x, delta_logp] integrates from eps to T on the device with the scipy-identical RK45
controller (inverse.ode), instead of scipy on a host copy.
"""
from __future__ import annotations

import numpy as np
import torch

from models import utils as mutils


def get_div_fn(fn):
    """Hutchinson-Skilling divergence estimate of fn (reference likelihood.py:26-37)."""

    def div_fn(x, t, eps):
        with torch.enable_grad():
            x.requires_grad_(True)
            fn_eps = torch.sum(fn(x, t) * eps)
            grad_fn_eps = torch.autograd.grad(fn_eps, x)[0]
        x.requires_grad_(False)
        return torch.sum(grad_fn_eps * eps, dim=tuple(range(1, len(x.shape))))

    return div_fn


def get_likelihood_fn(sde, inverse_scaler, hutchinson_type="Rademacher", rtol=1e-5, atol=1e-5,
                      method="RK45", eps=1e-5):
    from inverse.ode import solve_ivp_rk

    def drift_fn(model, x, t):
        score_fn = mutils.get_score_fn(sde, model, train=False, continuous=True)
        return sde.reverse(score_fn, probability_flow=True).sde(x, t)[0]

    def div_fn(model, x, t, noise):
        return get_div_fn(lambda xx, tt: drift_fn(model, xx, tt))(x, t, noise)

    def likelihood_fn(model, data):
        with torch.no_grad():
            shape = data.shape
            B = shape[0]
            if hutchinson_type == "Gaussian":
                epsilon = torch.randn_like(data)
            elif hutchinson_type == "Rademacher":
                epsilon = torch.randint_like(data, low=0, high=2).float() * 2 - 1.
            else:
                raise NotImplementedError(f"Hutchinson type {hutchinson_type} unknown.")

            def ode_func(t, x):
                sample = x[:-B].reshape(shape).to(torch.float32)
                vec_t = torch.ones(B, device=sample.device) * t
                drift = drift_fn(model, sample, vec_t).reshape(-1)
                logp_grad = div_fn(model, sample, vec_t, epsilon).reshape(-1)
                return torch.cat([drift.double(), logp_grad.double()])

            init = torch.cat([data.reshape(-1).double(),
                              torch.zeros(B, dtype=torch.float64, device=data.device)])
            with mutils.input_grad_only(model):
                sol = solve_ivp_rk(ode_func, (eps, sde.T), init, rtol=rtol, atol=atol,
                                   method=method)
            zp = sol.y
            z = zp[:-B].reshape(shape).to(torch.float32)
            delta_logp = zp[-B:].to(torch.float32)
            prior_logp = sde.prior_logp(z)
            bpd = -(prior_logp + delta_logp) / np.log(2)
            bpd = bpd / np.prod(shape[1:])
            offset = 7. - inverse_scaler(-1.)
            return bpd + offset, z, sol.nfev

    return likelihood_fn
