"""Conditional (inverse-problem) samplers: DPS and the controlled ODE sampler
(reference inverse/conditional_sampling.py:10-169).

Same factories and contracts: `get_sampler(config, obsv_sde, shape, lambda_schedule, eps)`
-> `sampler(model, z=None) -> x`; `config.inverse.sampler` in {'dps', 'controlled'},
`config.inverse.solver` in {'RK45', 'RK23', 'fixed'}.

MI355X design: the ODE state never leaves HBM.  The reference flattens the batch into a
float64 numpy vector for scipy's solve_ivp and copies it host<->device at every function
evaluation; here `inverse.ode.solve_ivp_rk` runs the identical RK45/RK23 controller on
device tensors (one scalar to the host per step).  The measurement operator is the
gather-form inpainting operator (no HW x HW matrices).  Batch sharding: each rank owns a
slice of the batch and of the observation; the two batch-global quantities -- the DPS
residual norm (conditional_sampling.py:129) and the solver's RMS error norms -- are
all-reduced (1 scalar each), so every rank takes the same step decisions.
"""
from __future__ import annotations

import torch

from models.utils import get_score_fn, input_grad_only
from . import ode


def _reduce_sumsq_fn(ctx):
    if ctx is None or not ctx.enabled:
        return None, 1

    def red(s):
        t = s.detach().reshape(1).to(torch.float64).clone()
        ctx.all_reduce_sum_(t)
        return t[0]

    return red, ctx.world_size


def get_solver(config, ode_func, x0, t1, shape, eps, ctx=None):
    """Integrate the sampler ODE from t1 down to eps (reference :10-30)."""
    solver = config.inverse.solver
    if solver in ("RK45", "RK23"):
        red, world = _reduce_sumsq_fn(ctx)
        n_global = x0.numel() * world
        sol = ode.solve_ivp_rk(ode_func, (t1, eps), x0, method=solver, rtol=1e-3, atol=1e-3,
                               reduce_sumsq=red, n_global=n_global,
                               max_steps=getattr(config.inverse, "max_steps", None))
        get_solver.last_nfe = sol.nfev
        return sol.y.reshape(shape).to(torch.float32)
    if solver == "fixed":
        x = x0.to(torch.float64).clone()
        dt = -.00002
        for t in torch.linspace(t1, eps, 5000):
            x += ode_func(t, x).to(torch.float64) * dt
        get_solver.last_nfe = 5000
        return x.reshape(shape).to(torch.float32)
    raise NotImplementedError(solver)


get_solver.last_nfe = 0


def get_sampler(config, obsv_sde, shape, lambda_schedule=lambda t: (1.0 - t) * 0.8, eps=1e-3,
                ctx=None):
    if config.inverse.sampler == "controlled":
        return get_controlled_sampler(config, obsv_sde, shape, lambda_schedule, eps=eps, ctx=ctx)
    if config.inverse.sampler == "dps":
        return get_dps_sampler(config, obsv_sde, shape, eps=eps, ctx=ctx)
    raise NotImplementedError(config.inverse.sampler)


def get_controlled_sampler(config, obsv_sde, shape, lambda_schedule, eps=1e-3, ctx=None):
    """Probability-flow ODE with the observed pixels pulled towards the noised observation
    (reference :40-97).  With A = diag(mask), L the observed-pixel selection:
        x <- w bcmm(L^T A, y_t) + (1 - w) bcmm(A, x) + bcmm(I - A, x)
    which in gather form is  w * scatter(y_t) + (1 - w) * mask * x + (1 - mask) * x."""
    device = config.device
    op = obsv_sde.operator

    def drift_fn(model, x, t):
        score_fn = get_score_fn(obsv_sde.state_sde, model, train=False, continuous=True)
        rsde = obsv_sde.state_sde.reverse(score_fn, probability_flow=True)
        return rsde.sde(x, t)[0]

    def optimize_fn(x, t):
        z = torch.randn_like(x)
        yt = obsv_sde.observe_sampling(z, t)
        w = lambda_schedule(t)[:, None, None, None]
        mask = op.mask.to(x.device)
        return w * op.transpose(yt, x.shape) + (1. - w) * (mask * x) + (1 - mask) * x

    def controlled_sampler(model, z=None):
        with torch.no_grad():
            x = obsv_sde.state_sde.prior_sampling(shape).to(device) if z is None else z

            def ode_func(t, xf):
                xh = xf.reshape(shape).to(torch.float32)
                vec_t = torch.ones(shape[0], device=device) * t
                xh = optimize_fn(xh, vec_t).reshape(shape)
                return drift_fn(model, xh, vec_t)

            return get_solver(config, ode_func, x.reshape(-1), obsv_sde.state_sde.T, shape, eps,
                              ctx=ctx)

    return controlled_sampler


def get_dps_sampler(config, obsv_sde, shape, eps=1e-3, ctx=None, noise=None):
    """Diffusion posterior sampling (reference :100-169).  `noise` optionally supplies the
    observation noise draw (default: torch.randn_like, as the reference)."""
    device = config.device
    obsv_var = config.inverse.variance
    y0 = obsv_sde.y0
    observation = y0 + (torch.randn_like(y0, device=device) if noise is None else noise) \
        * obsv_var ** .5
    red, _ = _reduce_sumsq_fn(ctx)
    sde = obsv_sde.state_sde

    def drift_fn(score, score_cond, x, t):
        drift, diffusion = sde.sde(x, t)
        return drift - diffusion[:, None, None, None] ** 2 * (score + score_cond) * 0.5

    def x0_hat_fn(model, xt, t):
        score = get_score_fn(sde, model, train=False, continuous=True)(xt, t)
        mean, std = sde.marginal_coef(t)
        return xt / mean[:, None, None, None] + std[:, None, None, None] ** 2 * score, score

    def cond_grad_fn(xt, x0_hat, scale=True):
        diff = observation - obsv_sde.operator(x0_hat, keep_shape=False)
        if red is None:
            norm = torch.linalg.norm(diff)
            logp = -norm ** 2 / obsv_var
        else:
            # ||diff|| over the whole (global) batch; the gradient of each shard's share of
            # -||diff||^2 / var depends only on that shard
            sumsq = torch.sum(diff * diff)
            norm = torch.sqrt(red(sumsq)).to(sumsq.dtype)
            logp = -sumsq / obsv_var
        g = torch.autograd.grad(outputs=logp, inputs=xt)[0]
        if scale is True:
            g = g / norm.detach()
        return g

    def make_ode_func(model):
        def ode_func(t, xf):
            xh = xf.reshape(shape).to(torch.float32).requires_grad_()
            vec_t = torch.ones(shape[0], device=device) * t
            x0_hat, score = x0_hat_fn(model, xh, vec_t)
            score_cond = cond_grad_fn(xh, x0_hat)
            return drift_fn(score.detach(), score_cond, xh.detach(), vec_t)
        return ode_func

    def dps_sampler(model, z=None):
        x = sde.prior_sampling(shape).to(device) if z is None else z
        with input_grad_only(model):
            return get_solver(config, make_ode_func(model), x.reshape(-1), sde.T, shape, eps,
                              ctx=ctx)

    dps_sampler.make_ode_func = make_ode_func
    dps_sampler.observation = observation
    return dps_sampler
