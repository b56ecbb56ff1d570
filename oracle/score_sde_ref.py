"""ORACLE (test infrastructure only) -- score-SDE engine restated on CPU.

SDE coefficients (reference sde_lib.py:136-307), the score wrapper
(models/utils.py:129-178), the PC samplers (sampling.py:176-411) and the DSM /
DDPM losses + Adam/EMA step (losses.py:29-224, models/ema.py:32-51), in plain
torch-CPU float32 with the reference's operation order.  Random draws are
INJECTED: every sampler takes an iterator of noise tensors consumed in the
reference's draw order, so a run can be replayed exactly against
tests/golden/pc_*.npz or against the GPU engine.
"""
from __future__ import annotations

import numpy as np
import torch


class SDESpec:
    """kind in {'vp', 'subvp', 've'} + its parameters and DDPM/SMLD tables."""

    def __init__(self, kind, N=1000, beta_min=0.1, beta_max=20., sigma_min=0.01, sigma_max=50.):
        self.kind, self.N = kind, N
        self.b0, self.b1 = beta_min, beta_max
        self.smin, self.smax = sigma_min, sigma_max
        if kind == "vp":
            self.betas = torch.linspace(beta_min / N, beta_max / N, N)
            self.alphas = 1. - self.betas
            self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
            self.sqrt_1m_ac = torch.sqrt(1. - self.alphas_cumprod)
            self.sqrt_ac = torch.sqrt(self.alphas_cumprod)
        if kind == "ve":
            self.sigmas = torch.exp(torch.linspace(np.log(sigma_min), np.log(sigma_max), N))

    T = 1

    def coefficient(self, t):
        if self.kind == "ve":
            sigma = self.smin * (self.smax / self.smin) ** t
            g = sigma * torch.sqrt(torch.tensor(2 * (np.log(self.smax) - np.log(self.smin))))
            return torch.zeros_like(t), g
        beta_t = self.b0 + t * (self.b1 - self.b0)
        if self.kind == "vp":
            return -0.5 * beta_t, torch.sqrt(beta_t)
        disc = 1. - torch.exp(-2 * self.b0 * t - (self.b1 - self.b0) * t ** 2)
        return -0.5 * beta_t, torch.sqrt(beta_t * disc)

    def drift(self, x, t):
        dc, _ = self.coefficient(t)
        return dc[:, None, None, None] if self.kind == "ve" else dc[:, None, None, None] * x

    def marginal_std(self, t):
        if self.kind == "ve":
            return self.smin * (self.smax / self.smin) ** t
        lm = -0.25 * t ** 2 * (self.b1 - self.b0) - 0.5 * t * self.b0
        if self.kind == "vp":
            return torch.sqrt(1. - torch.exp(2. * lm))
        return 1 - torch.exp(2. * lm)

    def marginal_mean_coef(self, t):
        lm = -0.25 * t ** 2 * (self.b1 - self.b0) - 0.5 * t * self.b0
        return torch.exp(lm)

    def index(self, t):
        return (t * (self.N - 1) / self.T).long()


def make_score(model_fn, sde: SDESpec, continuous):
    """models/utils.py:129-178."""

    def score(x, t):
        if sde.kind in ("vp", "subvp"):
            if continuous or sde.kind == "subvp":
                labels = t * 999
                out = model_fn(x, labels)
                std = sde.marginal_std(t)
            else:
                labels = t * (sde.N - 1)
                out = model_fn(x, labels)
                std = sde.sqrt_1m_ac[labels.long()]
            return -out / std[:, None, None, None]
        if continuous:
            labels = sde.marginal_std(t)
        else:
            labels = torch.round((sde.T - t) * (sde.N - 1)).long()
        return model_fn(x, labels)

    return score


def _predictor(name, sde, score, x, t, draw):
    if name == "none":
        return x, x
    if name == "euler_maruyama":  # sampling.py:181-187
        dt = -1. / sde.N
        z = draw()
        _, g = sde.coefficient(t)
        drift = sde.drift(x, t) - g[:, None, None, None] ** 2 * score(x, t) * 1.
        x_mean = x + drift * dt
        return x_mean + g[:, None, None, None] * np.sqrt(-dt) * z, x_mean
    if name == "reverse_diffusion":  # sampling.py:195-200 + sde_lib.py:112-117
        ts = sde.index(t)
        if sde.kind == "vp":
            f = torch.sqrt(sde.alphas[ts])[:, None, None, None] * x - x
            G = torch.sqrt(sde.betas[ts])
        elif sde.kind == "ve":
            sig = sde.sigmas[ts]
            adj = torch.where(ts == 0, torch.zeros_like(t), sde.sigmas[ts - 1])
            f = torch.zeros_like(x)
            G = torch.sqrt(sig ** 2 - adj ** 2)
        else:
            dt = 1 / sde.N
            f = sde.drift(x, t) * dt
            G = sde.coefficient(t)[1] * torch.sqrt(torch.tensor(dt))
        rev_f = f - G[:, None, None, None] ** 2 * score(x, t) * 1.
        z = draw()
        x_mean = x - rev_f
        return x_mean + G[:, None, None, None] * z, x_mean
    if name == "ancestral_sampling":  # sampling.py:211-233
        ts = sde.index(t)
        s = score(x, t)
        if sde.kind == "ve":
            sig = sde.sigmas[ts]
            adj = torch.where(ts == 0, torch.zeros_like(t), sde.sigmas[ts - 1])
            x_mean = x + s * (sig ** 2 - adj ** 2)[:, None, None, None]
            std = torch.sqrt((adj ** 2 * (sig ** 2 - adj ** 2)) / (sig ** 2))
            return x_mean + std[:, None, None, None] * draw(), x_mean
        beta = sde.betas[ts]
        x_mean = (x + beta[:, None, None, None] * s) / torch.sqrt(1. - beta)[:, None, None, None]
        return x_mean + torch.sqrt(beta)[:, None, None, None] * draw(), x_mean
    raise NotImplementedError(name)


def _corrector(name, sde, score, x, t, snr, n_steps, draw):
    if name == "none":
        return x, x
    alpha = sde.alphas[sde.index(t)] if sde.kind in ("vp", "subvp") else torch.ones_like(t)
    x_mean = x
    if name == "langevin":  # sampling.py:262-282
        for _ in range(n_steps):
            grad = score(x, t)
            noise = draw()
            gn = torch.norm(grad.reshape(grad.shape[0], -1), dim=-1).mean()
            nn_ = torch.norm(noise.reshape(noise.shape[0], -1), dim=-1).mean()
            step = (snr * nn_ / gn) ** 2 * 2 * alpha
            x_mean = x + step[:, None, None, None] * grad
            x = x_mean + torch.sqrt(step * 2)[:, None, None, None] * noise
        return x, x_mean
    if name == "ald":  # sampling.py:294-319
        std = sde.marginal_std(t)
        for _ in range(n_steps):
            grad = score(x, t)
            noise = draw()
            step = (snr * std) ** 2 * 2 * alpha
            x_mean = x + step[:, None, None, None] * grad
            x = x_mean + noise * torch.sqrt(step * 2)[:, None, None, None]
        return x, x_mean
    raise NotImplementedError(name)


def pc_sample(model_fn, sde: SDESpec, prior, predictor, corrector, snr, n_steps, continuous,
              denoise=True, eps=1e-3, draws=None, n_iters=None, on_step=None):
    """Reference get_pc_sampler loop (sampling.py:390-409) with injected noise.

    `draws`: iterator of noise tensors in the reference's draw order; None ->
    torch.randn_like.  Returns (samples, nfe)."""
    score = make_score(model_fn, sde, continuous)
    it = iter(draws) if draws is not None else None

    def draw_like(x):
        return (lambda: next(it)) if it is not None else (lambda: torch.randn_like(x))

    x = prior.clone()
    x_mean = x
    ts = torch.linspace(sde.T, eps, sde.N)
    n_iters = sde.N if n_iters is None else n_iters
    with torch.no_grad():
        for i in range(n_iters):
            vec_t = torch.ones(x.shape[0]) * ts[i]
            x, x_mean = _corrector(corrector, sde, score, x, vec_t, snr, n_steps, draw_like(x))
            x, x_mean = _predictor(predictor, sde, score, x, vec_t, draw_like(x))
            if on_step is not None:
                on_step(i, x, x_mean)
    return (x_mean if denoise else x), sde.N * (n_steps + 1)


def dsm_loss(model_fn, sde: SDESpec, batch, t, z, reduce_mean=True):
    """losses.py:87-113 (likelihood_weighting=False, continuous) with given t, z."""
    std = sde.marginal_std(t)
    mean = sde.marginal_mean_coef(t)[:, None, None, None] * batch
    perturbed = mean + std[:, None, None, None] * z
    score = make_score(model_fn, sde, True)(perturbed, t)
    losses = torch.square(score * std[:, None, None, None] + z)
    red = torch.mean if reduce_mean else (lambda v, dim: 0.5 * torch.sum(v, dim=dim))
    return torch.mean(red(losses.reshape(losses.shape[0], -1), dim=-1))


def ddpm_loss(model_fn, sde: SDESpec, batch, labels, noise, reduce_mean=True):
    """losses.py:142-162 with given labels / noise."""
    perturbed = sde.sqrt_ac[labels, None, None, None] * batch + \
        sde.sqrt_1m_ac[labels, None, None, None] * noise
    out = model_fn(perturbed, labels)
    losses = torch.square(out - noise)
    red = torch.mean if reduce_mean else (lambda v, dim: 0.5 * torch.sum(v, dim=dim))
    return torch.mean(red(losses.reshape(losses.shape[0], -1), dim=-1))
