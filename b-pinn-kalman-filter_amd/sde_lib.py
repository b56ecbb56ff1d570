"""SDE plugin surface (reference: sde_lib.py:7-307).

`SDE` keeps the reference's abstract interface so user SDEs drop in unchanged:
`T, sde, coefficient, marginal_coef, marginal_prob, prior_sampling, prior_logp`
and the optional `discretize`; `reverse(score_fn, probability_flow)` builds the
reverse-time SDE/ODE object.  VP / sub-VP / VE are the three concrete SDEs.

All coefficient formulas evaluate in the dtype/device of `t` with the same
float32 operation order as the reference, which is what lets the sampler
precompute per-step coefficient tables on the host (sampling.py) that are
bit-identical to what the reference computes per step.
"""
from __future__ import annotations

import abc

import numpy as np
import torch


class SDE(abc.ABC):
    """Forward SDE dx = f(x, t) dt + g(t) dW, evaluated on mini-batches."""

    def __init__(self, N):
        super().__init__()
        self.N = N  # number of discretisation steps

    @property
    @abc.abstractmethod
    def T(self):
        """End time."""

    @abc.abstractmethod
    def sde(self, x, t):
        """Return (drift, diffusion)."""

    @abc.abstractmethod
    def coefficient(self, t):
        """(drift coefficient, diffusion coefficient) of a linear SDE."""

    @abc.abstractmethod
    def marginal_coef(self, t):
        """(mean coefficient, std) of p_t(x | x_0)."""

    @abc.abstractmethod
    def marginal_prob(self, x, t):
        """(mean, std) of p_t(x | x_0)."""

    @abc.abstractmethod
    def prior_sampling(self, shape):
        """One sample of the prior p_T."""

    @abc.abstractmethod
    def prior_logp(self, z):
        """log p_T(z) per sample."""

    def discretize(self, x, t):
        """Euler-Maruyama discretisation x_{i+1} = x_i + f_i + G_i z_i (default)."""
        dt = 1 / self.N
        drift, diffusion = self.sde(x, t)
        return drift * dt, diffusion * torch.sqrt(torch.tensor(dt, device=t.device))

    def reverse(self, score_fn, probability_flow=False):
        """Reverse-time SDE (or probability-flow ODE) driven by `score_fn`."""
        return _ReverseSDE(self, score_fn, probability_flow)


class _ReverseSDE:
    """Reverse-time process of a forward SDE (reference sde_lib.py:81-119).

    The reference builds a subclass of the forward SDE's class on every call; a
    plain wrapper object carries the same interface (`N`, `T`, `sde`,
    `discretize`, `probability_flow`) and forwards everything else to the
    forward SDE, so isinstance-free code behaves identically.
    """

    def __init__(self, fwd: SDE, score_fn, probability_flow: bool):
        self._fwd = fwd
        self.N = fwd.N
        self.score_fn = score_fn
        self.probability_flow = probability_flow

    @property
    def T(self):
        return self._fwd.T

    def __getattr__(self, name):
        return getattr(self._fwd, name)

    def _weight(self):
        return 0.5 if self.probability_flow else 1.

    def sde(self, x, t):
        drift, diffusion = self._fwd.sde(x, t)
        score = self.score_fn(x, t)
        drift = drift - diffusion[:, None, None, None] ** 2 * score * self._weight()
        return drift, (0. if self.probability_flow else diffusion)

    def discretize(self, x, t):
        f, G = self._fwd.discretize(x, t)
        rev_f = f - G[:, None, None, None] ** 2 * self.score_fn(x, t) * self._weight()
        rev_G = torch.zeros_like(G) if self.probability_flow else G
        return rev_f, rev_G


def _gaussian_prior_logp(z, scale2=1.0):
    n = np.prod(z.shape[1:])
    return -n / 2. * np.log(2 * np.pi * scale2) - torch.sum(z ** 2, dim=(1, 2, 3)) / (2. * scale2)


class VPSDE(SDE):
    """Variance-preserving SDE, beta(t) linear in t (reference sde_lib.py:136-199)."""

    def __init__(self, beta_min=0.1, beta_max=20, N=1000):
        super().__init__(N)
        self.beta_0 = beta_min
        self.beta_1 = beta_max
        # DDPM tables, float32 (reference :149-153)
        self.discrete_betas = torch.linspace(beta_min / N, beta_max / N, N)
        self.alphas = 1. - self.discrete_betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.sqrt_alphas_cumprod = torch.sqrt(self.alphas_cumprod)
        self.sqrt_1m_alphas_cumprod = torch.sqrt(1. - self.alphas_cumprod)

    @property
    def T(self):
        return 1

    def coefficient(self, t):
        beta_t = self.beta_0 + t * (self.beta_1 - self.beta_0)
        return -0.5 * beta_t, torch.sqrt(beta_t)

    def sde(self, x, t):
        dc, gc = self.coefficient(t)
        return dc[:, None, None, None] * x, gc

    def marginal_coef(self, t):
        log_mean = -0.25 * t ** 2 * (self.beta_1 - self.beta_0) - 0.5 * t * self.beta_0
        return torch.exp(log_mean), torch.sqrt(1. - torch.exp(2. * log_mean))

    def marginal_prob(self, x, t):
        mean, std = self.marginal_coef(t)
        return mean[:, None, None, None] * x, std

    def prior_sampling(self, shape):
        return torch.randn(*shape)

    def prior_logp(self, z):
        return _gaussian_prior_logp(z)

    def timestep_index(self, t):
        """Integer DDPM step of continuous t: (t * (N - 1) / T).long() (reference :193)."""
        return (t * (self.N - 1) / self.T).long()

    def discretize(self, x, t):
        ts = self.timestep_index(t)
        beta = self.discrete_betas.to(x.device)[ts]
        alpha = self.alphas.to(x.device)[ts]
        f = torch.sqrt(alpha)[:, None, None, None] * x - x
        return f, torch.sqrt(beta)


class subVPSDE(SDE):
    """sub-VP SDE (reference sde_lib.py:202-250)."""

    def __init__(self, beta_min=0.1, beta_max=20, N=1000):
        super().__init__(N)
        self.beta_0 = beta_min
        self.beta_1 = beta_max

    @property
    def T(self):
        return 1

    def coefficient(self, t):
        beta_t = self.beta_0 + t * (self.beta_1 - self.beta_0)
        discount = 1. - torch.exp(-2 * self.beta_0 * t - (self.beta_1 - self.beta_0) * t ** 2)
        return -0.5 * beta_t, torch.sqrt(beta_t * discount)

    def sde(self, x, t):
        dc, gc = self.coefficient(t)
        return dc[:, None, None, None] * x, gc

    def marginal_coef(self, t):
        log_mean = -0.25 * t ** 2 * (self.beta_1 - self.beta_0) - 0.5 * t * self.beta_0
        return torch.exp(log_mean), 1 - torch.exp(2. * log_mean)

    def marginal_prob(self, x, t):
        mean, std = self.marginal_coef(t)
        return mean[:, None, None, None] * x, std

    def prior_sampling(self, shape):
        return torch.randn(*shape)

    def prior_logp(self, z):
        return _gaussian_prior_logp(z)


class VESDE(SDE):
    """Variance-exploding SDE (reference sde_lib.py:253-307)."""

    def __init__(self, sigma_min=0.01, sigma_max=50, N=1000):
        super().__init__(N)
        self.sigma_min = sigma_min
        self.sigma_max = sigma_max
        self.discrete_sigmas = torch.exp(torch.linspace(np.log(sigma_min), np.log(sigma_max), N))

    @property
    def T(self):
        return 1

    def coefficient(self, t):
        sigma = self.sigma_min * (self.sigma_max / self.sigma_min) ** t
        rate = torch.sqrt(torch.tensor(2 * (np.log(self.sigma_max) - np.log(self.sigma_min)),
                                       device=t.device))
        return torch.zeros_like(t), sigma * rate

    def sde(self, x, t):
        dc, gc = self.coefficient(t)
        return dc[:, None, None, None], gc

    def marginal_coef(self, t):
        return torch.ones_like(t), self.sigma_min * (self.sigma_max / self.sigma_min) ** t

    def marginal_prob(self, x, t):
        return x, self.sigma_min * (self.sigma_max / self.sigma_min) ** t

    def prior_sampling(self, shape):
        return torch.randn(*shape) * self.sigma_max

    def prior_logp(self, z):
        return _gaussian_prior_logp(z, self.sigma_max ** 2)

    def timestep_index(self, t):
        return (t * (self.N - 1) / self.T).long()

    def discretize(self, x, t):
        ts = self.timestep_index(t)
        sigma = self.discrete_sigmas.to(t.device)[ts]
        adj = torch.where(ts == 0, torch.zeros_like(t), self.discrete_sigmas[ts - 1].to(t.device))
        return torch.zeros_like(x), torch.sqrt(sigma ** 2 - adj ** 2)


class OBSVSDE(SDE):
    """Observation process y_t of a hidden state SDE (reference sde_lib.py:122-133)."""

    def __init__(self, N, y0, operator):
        super().__init__(N)
        self.y0 = y0
        self.operator = operator

    @abc.abstractmethod
    def observe_sampling(self, z, t):
        """y_t sample given standard-normal state noise z."""


class LOBSVSDE(OBSVSDE):
    """Linear observation y = A x of a state SDE (reference sde_lib.py:310-359).

    `observe_sampling(z, t) = alpha(t) y0 + beta(t) A z` with (alpha, beta) the state SDE's
    marginal coefficients.  A is the operator's gather form (inverse/operators.py); the
    reference's dense `to_matrix` / `mat & mat` covariance (:327-334) is not materialised.
    """

    def __init__(self, state_sde: SDE, y0, operator):
        super().__init__(state_sde.N, y0, operator)
        self.state_sde = state_sde
        self.mat = None

    def observe_sampling(self, z, t):
        alpha, beta = self.state_sde.marginal_coef(t)
        return alpha[:, None, None] * self.y0 + beta[:, None, None] * self.operator(z, False)

    def prior_sampling(self, shape):
        return None

    @property
    def T(self):
        return 1

    def marginal_prob(self, z, t):
        raise NotImplementedError("LOBSVSDE.marginal_prob needs the dense observation matrix")

    def prior_logp(self, z):
        return None

    def sde(self, x, t):
        return None

    def coefficient(self, t):
        return None

    def marginal_coef(self, t):
        return None
