"""PINN = FlowNet + PressureNet + Navier-Stokes residual (reference: pinn_kalman/pinn.py:34-114).

`PINN(config)`; `forward(f1, f2, x, y, t, size=None) -> (cascaded_flow, pressure)`;
`equation_mse(x, y, t, flow, pres, Re)`; `step(ft, u)`.  The residual is the
reference's: derivatives are autograd sensitivities of the predicted fields with
respect to the coordinate INPUT channels x, y (per pixel) and t (per sample) --
first order with create_graph (so they train the nets), second order without
(SURVEY.md Appendix A.5-6).  The second derivative through the warping runs on
the HIP grid_sample grad2 kernel.

Only the deterministic PINN is built: B_PINN needs `bayesian_torch` (unpinned,
absent here) and is out of scope.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from models.flownet import FlowNet, PressureNet, project

# diagnostics hook (tools/prof_pinn_phases.py): called with a phase name between the residual's
# derivative passes; None in normal use
PHASE_MARK = None


def _mark(name):
    if PHASE_MARK is not None:
        PHASE_MARK(name)


def fd_residual_mse(u, v, p, u_t, v_t, h, Re):
    """MSEs of the x/y momentum and mass residuals with spatial derivatives on the ns_step
    stencil (reference diff_x / diff_y, op/ns_step_kernel.cu:50-75): u, v, p [B, 1, H, W],
    u_t, v_t [B], grid spacing h.  Second derivatives are the stencil applied twice."""
    from op.ns_step import stencil_gradient
    u_x, u_y = stencil_gradient(u, h)
    v_x, v_y = stencil_gradient(v, h)
    p_x, p_y = stencil_gradient(p, h)
    u_xx = stencil_gradient(u_x, h)[0]
    u_yy = stencil_gradient(u_y, h)[1]
    v_xx = stencil_gradient(v_x, h)[0]
    v_yy = stencil_gradient(v_y, h)[1]
    u_t = u_t[:, None, None, None]
    v_t = v_t[:, None, None, None]
    nu = 1.0 / Re
    res_x = u_t + (u * u_x + v * u_y) + p_x - nu * (u_xx + u_yy)
    res_y = v_t + (u * v_x + v * v_y) + p_y - nu * (v_xx + v_yy)
    res_mass = u_x + v_y
    return (res_x ** 2).mean() + (res_y ** 2).mean() + (res_mass ** 2).mean()


def get_model(config):
    arch = config.model.arch
    if arch == "flownet":
        return FlowNet(config)
    raise NotImplementedError(f"PINN flow architecture {arch!r} is not built "
                              "(only 'flownet' is on the hot path)")


class PINN(nn.Module):
    """Input (f1, f2) frames [B, C, N, N], coordinate channels x, y [B, 1, N, N], t [B];
    output (cascaded flow list, pressure [B, 1, N, N])."""

    def __init__(self, config):
        super().__init__()
        self.device = config.device
        self.dt = config.data.dt
        self.flownet = get_model(config).to(self.device)
        self.pressurenet = PressureNet(config).to(self.device)
        mask_u, mask_v = self.get_mask(config)
        # non-persistent buffers: they follow .to(device) and stay out of the state dict
        self.register_buffer("mask_u", mask_u, persistent=False)
        self.register_buffer("mask_v", mask_v, persistent=False)

    def get_mask(self, config):
        """[2, N, N] selectors of u and v ("differentiable slicing", reference pinn.py:50-61)."""
        n = config.data.image_size
        one, zero = torch.ones(n, n), torch.zeros(n, n)
        return (torch.stack([one, zero]).to(config.device),
                torch.stack([zero, one]).to(config.device))

    def forward(self, f1, f2, x, y, t, size=None):
        flow = self.flownet(f1, f2, x, y, t, size=size)
        return flow, self.pressurenet(flow, x, y, t)

    def advection_mse(self, x, y, t, prediction):
        return None

    def equation_mse(self, x, y, t, flow, pres, Re):
        """Sum of the MSEs of the x/y momentum and mass residuals (reference pinn.py:72-111)."""
        u = (self.mask_u * flow).sum(dim=1).unsqueeze(1)
        v = (self.mask_v * flow).sum(dim=1).unsqueeze(1)
        p = pres
        grad = torch.autograd.grad
        _mark("d1_u")
        u_x, u_y, u_t = grad(u.sum(), (x, y, t), create_graph=True, retain_graph=True)
        _mark("d1_v")
        v_x, v_y, v_t = grad(v.sum(), (x, y, t), create_graph=True, retain_graph=True)
        _mark("d1_p")
        p_x, p_y = grad(p.sum(), (x, y), create_graph=True, retain_graph=True)
        _mark("d2")
        u_xx = grad(u_x.sum(), x, retain_graph=True)[0]
        u_yy = grad(u_y.sum(), y, retain_graph=True)[0]
        v_xx = grad(v_x.sum(), x, retain_graph=True)[0]
        v_yy = grad(v_y.sum(), y, retain_graph=True)[0]
        _mark("residual")
        u_t = u_t[:, None, None, None]
        v_t = v_t[:, None, None, None]
        nu = 1.0 / Re
        res_x = u_t + (u * u_x + v * u_y) + p_x - nu * (u_xx + u_yy)
        res_y = v_t + (u * v_x + v * v_y) + p_y - nu * (v_xx + v_yy)
        res_mass = u_x + v_y
        mse = torch.nn.MSELoss()
        zeros = torch.zeros_like(x)
        return mse(res_x, zeros) + mse(res_y, zeros) + mse(res_mass, zeros)

    def equation_mse_fd(self, x, y, t, flow, pres, Re, h=None):
        """Navier-Stokes residual with SPATIAL derivatives on the ns_step stencil (the
        reference's diff_x / diff_y, op/ns_step_kernel.cu:50-75, run by the same HIP
        kernel as the simulator) instead of autograd input sensitivities; u_t, v_t stay
        autograd derivatives w.r.t. t as in `equation_mse`.  `h` is the grid spacing
        (default: the mean spacing of the x coordinate channel along the width).
        Differentiable to any order (the stencil's backward is its adjoint kernel)."""
        u = (self.mask_u * flow).sum(dim=1).unsqueeze(1)
        v = (self.mask_v * flow).sum(dim=1).unsqueeze(1)
        p = pres
        if h is None:
            h = float((x[:, :, :, -1] - x[:, :, :, 0]).mean()) / (x.shape[-1] - 1)
        u_t = torch.autograd.grad(u.sum(), t, create_graph=True, retain_graph=True)[0]
        v_t = torch.autograd.grad(v.sum(), t, create_graph=True, retain_graph=True)[0]
        return fd_residual_mse(u, v, p, u_t, v_t, h, Re)

    def step(self, ft, u):
        """Advance a field by the predicted flow (reference pinn.py:113-114)."""
        return project(ft, u, self.dt)
