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

    def forward_residual_copies(self, f1, f2, x, y, t, Re, copies=4):
        """forward() and equation_mse() together, with the residual's derivative passes
        batched over copies of the inputs: (cascaded flows, pressure, residual MSE), the same
        values and parameter gradients as forward() + equation_mse() (reference pinn.py:72-111).

        equation_mse differentiates the nets seven times with autograd.grad -- u, v and p
        w.r.t. (x, y, t), then u_x, u_y, v_x, v_y w.r.t. x or y -- each pass a few hundred
        small launches (FlowNet at 64^2 runs ~8 samples per launch on a rank of the 8-GPU
        point: launch-bound).  Here FlowNet runs once on `copies` stacked copies of the batch,
        each copy with its own coordinate tensors, and ONE first-order pass takes the
        cotangent u on some copies and v on the others (samples never interact -- x.max() is
        taken per copy, layers.spatial_groups -- so copy c's input gradient is exactly the
        derivative of its own selected field):
          copies = 4: u, u, v, v -- one second-order pass takes u_x on copy 0, u_y on copy 1,
                      v_x on copy 2, v_y on copy 3, i.e. u_xx, u_yy, v_xx, v_yy at once;
          copies = 2: u, v -- two second-order passes (w.r.t. x, then w.r.t. y).
        PressureNet (its flow input is detached, reference flownet.py:286) runs once, on its
        own view of x, y, inside the same first-order pass.  The data losses read copy 0.
        More FLOPs (FlowNet forward x copies), far fewer launches: the form for small
        per-GPU batches (losses.get_pinn_step_fn picks it)."""
        from models import layers
        from op import channels
        assert copies in (2, 4)
        B = x.shape[0]
        sel = (0, 0, 1, 1) if copies == 4 else (0, 1)  # flow channel of each copy's cotangent
        rep = lambda v: channels.cat([v] * copies, 0)  # noqa: E731  (backward: one split)
        X, Y, T = rep(x), rep(y), rep(t)
        xp, yp = x.view_as(x), y.view_as(y)  # PressureNet's own handles on x, y
        with layers.spatial_groups(copies):
            flows = self.flownet(f1.repeat(copies, 1, 1, 1), f2.repeat(copies, 1, 1, 1), X, Y, T)
        flow0 = [channels.split(f, (B,) * copies, 0)[0] for f in flows]
        pres = self.pressurenet(flow0, xp, yp, t)
        ff = flows[-1]
        w, wx, wy = self._copy_weights(copies, sel, ff.device)
        cot = (ff.view((copies, B) + tuple(ff.shape[1:])) * w[:, None]).sum()
        grad = torch.autograd.grad
        _mark("d1")
        gX, gY, gT, p_x, p_y = grad(cot + pres.sum(), (X, Y, T, xp, yp), create_graph=True,
                                    retain_graph=True)
        gXs = channels.split(gX, (B,) * copies, 0)
        gYs = channels.split(gY, (B,) * copies, 0)
        gTs = channels.split(gT, (B,) * copies, 0)
        cu, cv = sel.index(0), sel.index(1)
        u_x, u_y, u_t = gXs[cu], gYs[cu], gTs[cu]
        v_x, v_y, v_t = gXs[cv], gYs[cv], gTs[cv]
        _mark("d2")
        if copies == 4:  # u_x on copy 0, u_y on 1, v_x on 2, v_y on 3: one pass
            l2 = ((gX.view((4, B) + tuple(gX.shape[1:])) * wx).sum()
                  + (gY.view((4, B) + tuple(gY.shape[1:])) * wy).sum())
            gX2, gY2 = grad(l2, (X, Y), retain_graph=True)
            gX2 = gX2.view((4, B) + tuple(gX2.shape[1:]))
            gY2 = gY2.view((4, B) + tuple(gY2.shape[1:]))
            u_xx, u_yy, v_xx, v_yy = gX2[0], gY2[1], gX2[2], gY2[3]
        else:
            gX2 = grad(gX.sum(), X, retain_graph=True)[0]
            gY2 = grad(gY.sum(), Y, retain_graph=True)[0]
            u_xx, v_xx = gX2[:B], gX2[B:]
            u_yy, v_yy = gY2[:B], gY2[B:]
        _mark("residual")
        u = flow0[-1][:, 0:1]
        v = flow0[-1][:, 1:2]
        u_t = u_t[:, None, None, None]
        v_t = v_t[:, None, None, None]
        nu = 1.0 / Re
        res_x = u_t + (u * u_x + v * u_y) + p_x - nu * (u_xx + u_yy)
        res_y = v_t + (u * v_x + v * v_y) + p_y - nu * (v_xx + v_yy)
        res_mass = u_x + v_y
        mse = torch.nn.MSELoss()
        zeros = torch.zeros_like(x)
        return flow0, pres, mse(res_x, zeros) + mse(res_y, zeros) + mse(res_mass, zeros)

    def _copy_weights(self, copies, sel, device):
        """(cotangent selector [copies, 2, 1, 1], x- and y-pass selectors [copies, 1, 1, 1, 1]) as
        cached device tensors: built on the first (eager) call, read by a captured step (no
        host-to-device copy inside a capture)."""
        cache = self.__dict__.setdefault("_copy_w", {})
        key = (copies, str(device))
        if key not in cache:
            w = torch.zeros(copies, 2, 1, 1)
            for c, ch in enumerate(sel):
                w[c, ch] = 1.0
            wx = torch.tensor([1.0, 0.0] * (copies // 2)).view(copies, 1, 1, 1, 1)
            cache[key] = (w.to(device), wx.to(device), (1.0 - wx).to(device))
        return cache[key]

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
