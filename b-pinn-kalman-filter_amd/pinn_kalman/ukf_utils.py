"""UKF dynamics on the ns_step stencil (reference pinn_kalman/ukf_utils.py:8-119).

The reference's square-root UKF (`torchfilter`, unpinned and absent here) is out of
scope; what it calls on the hot path is built: `patch` / `unpatch` (the state layout of
p x p field patches) and `NSDynamics.forward`, which advances the unpatched fields by one
simulator step -- update_velocity, update_pressure, update_density (ukf_utils.py:109-111)
-- here the fused `ns_step.full_step` (bit-identical to the three calls), and returns
the re-patched state with the reference's constant process covariance 1e-8 I.
`NSDynamics` is a plain nn.Module with the torchfilter `DynamicsModel` call contract
(`state_dim`, `forward(initial_states, controls) -> (states, covariance)`); the debug
prints of the reference (NaN/inf checks, each a device sync) are dropped.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from op import ns_step

DT = 0.0005 * 5  # reference ukf_utils.py:105-106 (the simulator's dt / dx)
DX = 1 / 200


def patch(x, p_size):
    """[B, C, H, W] -> [C * B * (H/p) * (W/p), p * p]: rows ordered (channel, sample,
    patch row, patch col) (reference ukf_utils.py:8-15)."""
    x = x.transpose(0, 1)
    x = x.unfold(2, p_size, p_size).unfold(3, p_size, p_size)
    return x.reshape(-1, p_size ** 2)


def unpatch(x, p_size, f_size, channel_num=6):
    """Inverse of `patch` (reference ukf_utils.py:17-22, which tiles the patches with
    torchvision's make_grid(nrow=f_size/p_size, padding=0)): -> [B, channel_num, f, f]."""
    num = f_size // p_size
    x = x.reshape(channel_num, -1, num, num, p_size, p_size)  # (c, b, i, j, a, b')
    x = x.permute(0, 1, 2, 4, 3, 5).reshape(channel_num, -1, f_size, f_size)
    return x.transpose(0, 1)


class NSDynamics(nn.Module):
    """Navier-Stokes dynamics of the patched UKF state (reference ukf_utils.py:85-119):
    channels (f, v, v, p) of [B, 4, S, S] fields, state rows of p * p values."""

    def __init__(self, config):
        super().__init__()
        self.dim = config.kf.patch_size
        self.size = config.data.image_size
        assert self.size % self.dim == 0
        self.state_dim = self.dim ** 2

    def unpatch(self, x):
        return unpatch(x, self.dim, self.size, 4)

    def forward(self, initial_states, controls=None):
        u = self.unpatch(initial_states)
        f, v, p = u[:, 0:1].contiguous(), u[:, 1:3].contiguous(), u[:, 3:4].contiguous()
        f, v, p = ns_step.full_step(f, v, p, DT, DX)
        state = patch(torch.cat([f, v, p], dim=1), self.dim)
        uncer = torch.eye(self.dim ** 2, device=state.device).unsqueeze(0).repeat(
            state.shape[0], 1, 1) * 1e-8
        return state, uncer
