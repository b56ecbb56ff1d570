"""Model registry, score-function wrappers (reference: models/utils.py:27-187).

`@register_model(name=)`, `get_model`, `create_model`, `get_model_fn` and
`get_score_fn` keep the reference's contracts.  Two MI355X-side changes:

* `create_model` does not wrap in `nn.DataParallel` (one process per GPU; the
  data-parallel path is `torch.distributed` + RCCL, see dist.py).  It wraps the
  network in `ModelHolder`, whose single child is called `module`, so state-dict
  keys keep the reference's `module.` prefix and reference checkpoints load.
* `get_score_fn` returns a `ScoreFn` object: calling it gives exactly the
  reference score; its `labels()`/`divisor()` pieces let the fused PC-sampler
  kernels fold "-model/std" into the update instead of materialising the score.
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch
import torch.nn as nn

import sde_lib

_MODELS: dict = {}


def register_model(cls=None, *, name=None):
    def _register(c):
        key = c.__name__ if name is None else name
        if key in _MODELS:
            raise ValueError(f"Already registered model with name: {key}")
        _MODELS[key] = c
        return c

    return _register if cls is None else _register(cls)


def get_model(name):
    return _MODELS[name]


def get_sigmas(config):
    """Geometric noise levels sigma_max -> sigma_min (reference :46-55)."""
    return np.exp(np.linspace(np.log(config.model.sigma_max), np.log(config.model.sigma_min),
                              config.model.num_scales))


def get_ddpm_params(config):
    """DDPM beta schedule in float64 (reference :58-84)."""
    T = 1000
    beta_start = config.model.beta_min / config.model.num_scales
    beta_end = config.model.beta_max / config.model.num_scales
    betas = np.linspace(beta_start, beta_end, T, dtype=np.float64)
    alphas = 1. - betas
    ac = np.cumprod(alphas, axis=0)
    return {"betas": betas, "alphas": alphas, "alphas_cumprod": ac,
            "sqrt_alphas_cumprod": np.sqrt(ac), "sqrt_1m_alphas_cumprod": np.sqrt(1. - ac),
            "beta_min": beta_start * (T - 1), "beta_max": beta_end * (T - 1),
            "num_diffusion_timesteps": T}


class ModelHolder(nn.Module):
    """Key-compatible stand-in for the reference's DataParallel wrapper."""

    def __init__(self, module):
        super().__init__()
        self.module = module

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)


def create_model(config, wrap=True):
    model = get_model(config.model.name)(config)
    model = model.to(config.device)
    return ModelHolder(model) if wrap else model


@contextlib.contextmanager
def input_grad_only(model):
    """Freeze the parameters for the duration (restored after): samplers that only need
    gradients w.r.t. the INPUT (DPS, the likelihood's divergence) then skip every
    weight-gradient kernel in backward.  Values are unchanged -- the reference computes the
    same input gradients with the parameters still requiring grad."""
    flags = [(p, p.requires_grad) for p in model.parameters()]
    for p, _ in flags:
        p.requires_grad_(False)
    try:
        yield model
    finally:
        for p, f in flags:
            p.requires_grad_(f)


def get_model_fn(model, train=False):
    def model_fn(x, labels):
        model.train(train)
        return model(x, labels)

    return model_fn


class ScoreFn:
    """score(x, t) exactly as the reference's closure (models/utils.py:129-178).

    VP / sub-VP: score = -model(x, labels) / std, with labels = 999 t (continuous or
    sub-VP) or t (N - 1) (discrete; std from sqrt_1m_alphas_cumprod[labels.long()]).
    VE: score = model(x, labels), labels = sigma(t) (continuous) or
    round((T - t)(N - 1)).long() (discrete).
    """

    def __init__(self, sde, model, train=False, continuous=False):
        if not isinstance(sde, (sde_lib.VPSDE, sde_lib.subVPSDE, sde_lib.VESDE)):
            raise NotImplementedError(f"SDE class {sde.__class__.__name__} not yet supported.")
        self.sde = sde
        self.model = model
        self.train = train
        self.continuous = continuous
        self.model_fn = get_model_fn(model, train=train)
        self.divides = not isinstance(sde, sde_lib.VESDE)

    def labels(self, t):
        sde = self.sde
        if self.divides:
            if self.continuous or isinstance(sde, sde_lib.subVPSDE):
                return t * 999
            return t * (sde.N - 1)
        if self.continuous:
            return sde.marginal_prob(torch.zeros_like(t), t)[1]
        lab = sde.T - t
        lab *= sde.N - 1
        return torch.round(lab).long()

    def divisor(self, t):
        """Per-sample std the model output is divided by (None for VE)."""
        sde = self.sde
        if not self.divides:
            return None
        if self.continuous or isinstance(sde, sde_lib.subVPSDE):
            return sde.marginal_coef(t)[1]
        lab = t * (sde.N - 1)
        return sde.sqrt_1m_alphas_cumprod.to(lab.device)[lab.long()]

    def __call__(self, x, t):
        out = self.model_fn(x, self.labels(t))
        if not self.divides:
            return out
        return -out / self.divisor(t)[:, None, None, None]


def get_score_fn(sde, model, train=False, continuous=False):
    return ScoreFn(sde, model, train=train, continuous=continuous)


def to_flattened_numpy(x):
    return x.detach().cpu().numpy().reshape((-1,))


def from_flattened_numpy(x, shape):
    return torch.from_numpy(x.reshape(shape))
