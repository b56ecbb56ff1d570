"""Inverse pipeline helpers on the hot path (reference inverse/inverse_lib.py:24-51)."""
from __future__ import annotations

import sde_lib


def get_sde(config):
    """run_lib._get_sde (reference run_lib.py:45-58)."""
    name = config.training.sde.lower()
    if name == "vpsde":
        return sde_lib.VPSDE(beta_min=config.model.beta_min, beta_max=config.model.beta_max,
                             N=config.model.num_scales), 1e-3
    if name == "subvpsde":
        return sde_lib.subVPSDE(beta_min=config.model.beta_min, beta_max=config.model.beta_max,
                                N=config.model.num_scales), 1e-3
    if name == "vesde":
        return sde_lib.VESDE(sigma_min=config.model.sigma_min, sigma_max=config.model.sigma_max,
                             N=config.model.num_scales), 1e-5
    raise NotImplementedError(f"SDE {config.training.sde} unknown.")


def get_obsvsde(config, y0, operator):
    sde, eps = get_sde(config)
    if config.inverse.sampler in ("controlled", "dps"):
        return sde_lib.LOBSVSDE(sde, y0, operator), eps
    raise NotImplementedError(config.inverse.sampler)
