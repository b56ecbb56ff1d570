"""`op.ns_step` -- 2-D Navier-Stokes explicit step on the HIP stencil (csrc/ns_step.hip).

Reference API: op/ns_step.py:19-26 -> ns_step_forward.update_{density,velocity,
pressure}(tensor, tensor, float dt, float dx) (op/ns_step.cpp:45-102); forward
only, no autograd, out-of-place.

`compat=True` (default, = reference behaviour) reproduces the unbind-stride quirk
of update_velocity (op/ns_step.cpp:70): for batch >= 2 the u / v views of the
intermediate velocity are read with batch stride H*W, so sample b advects memory
plane b (u) / b+1 (v) of vel_n.  `compat=False` advects the intended planes.

Other reference properties kept: H == W is not required but the plane is indexed
as the reference does (contiguous axis = size(2)); a velocity component exactly
0 produces NaN (CIP divides by sign(u)); dt / dx are rounded to float32.
Lifted: the reference maps the batch to threadIdx.x (B <= 1024); any B works here.
"""
from __future__ import annotations

import torch

from ._lib import check, lib, require_hip, stream_ptr


def _check(name, *ts):
    require_hip(*ts, what=f"ns_step.{name}")
    for t in ts:
        if t.dtype != torch.float32:
            raise RuntimeError(f"ns_step.{name}: float32 tensors required, got {t.dtype}")
        if t.ndim != 4:
            raise RuntimeError(f"ns_step.{name}: expected [B, C, H, W] tensors")


def _geo(t):
    B, _, nx, ny = t.shape  # reference: gridDim.x = size(2), gridDim.y = size(3)
    return B, nx, ny


def _workspace(op, B, nx, ny, device):
    nbytes = lib.bpk_ns_workspace_bytes(op, B, nx, ny)
    return torch.empty(max(nbytes // 4, 1), device=device, dtype=torch.float32)


def update_density(dens, vel, dt, dx):
    _check("update_density", dens, vel)
    dens, vel = dens.contiguous(), vel.contiguous()
    B, nx, ny = _geo(dens)
    out = torch.empty_like(dens)
    ws = _workspace(0, B, nx, ny, dens.device)
    check(lib.bpk_ns_update_density_f32(dens.data_ptr(), vel.data_ptr(), out.data_ptr(),
                                        ws.data_ptr(), B, nx, ny, float(dt), float(dx),
                                        stream_ptr(dens.device)), "ns_step.update_density")
    return out


def update_velocity(vel, pres, dt, dx, compat=True):
    _check("update_velocity", vel, pres)
    vel, pres = vel.contiguous(), pres.contiguous()
    B, nx, ny = _geo(vel)
    out = torch.empty_like(vel)
    ws = _workspace(1, B, nx, ny, vel.device)
    check(lib.bpk_ns_update_velocity_f32(vel.data_ptr(), pres.data_ptr(), out.data_ptr(),
                                         ws.data_ptr(), B, nx, ny, float(dt), float(dx),
                                         int(bool(compat)), stream_ptr(vel.device)),
          "ns_step.update_velocity")
    return out


def update_pressure(pres, vel, dt, dx):
    _check("update_pressure", pres, vel)
    pres, vel = pres.contiguous(), vel.contiguous()
    B, nx, ny = _geo(pres)
    out = torch.empty_like(pres)
    check(lib.bpk_ns_update_pressure_f32(pres.data_ptr(), vel.data_ptr(), out.data_ptr(), B, nx,
                                         ny, float(dt), float(dx), stream_ptr(pres.device)),
          "ns_step.update_pressure")
    return out


def full_step(dens, vel, pres, dt, dx, compat=True, out=None):
    """One simulator step (pinn_kalman/simulator.py:55-57) in two fused launches:
    vel' = update_velocity(vel, pres); pres' = update_pressure(pres, vel');
    dens' = update_density(dens, vel').  Bit-identical to the three calls."""
    _check("full_step", dens, vel, pres)
    dens, vel, pres = dens.contiguous(), vel.contiguous(), pres.contiguous()
    B, nx, ny = _geo(dens)
    if out is None:
        out = (torch.empty_like(dens), torch.empty_like(vel), torch.empty_like(pres))
    d1, v1, p1 = out
    check(lib.bpk_ns_full_step_f32(dens.data_ptr(), vel.data_ptr(), pres.data_ptr(), d1.data_ptr(),
                                   v1.data_ptr(), p1.data_ptr(), None, B, nx, ny, float(dt),
                                   float(dx), int(bool(compat)), stream_ptr(dens.device)),
          "ns_step.full_step")
    return d1, v1, p1


# low-level kernels (one launch each), exposed for tests and custom pipelines
def gradient(field, dx):
    _check("gradient", field)
    f = field.contiguous()
    if f.shape[1] != 1:
        raise RuntimeError("ns_step.gradient: expects a [B, 1, H, W] scalar field")
    B, nx, ny = _geo(f)
    fx, fy = torch.empty_like(f), torch.empty_like(f)
    check(lib.bpk_ns_gradient_f32(f.data_ptr(), nx * ny, fx.data_ptr(), fy.data_ptr(),
                                  B, nx, ny, float(dx), stream_ptr(f.device)), "ns_step.gradient")
    return fx, fy


def gradient_adjoint(gx, gy, dx):
    """Dx^T gx + Dy^T gy for the stencil of `gradient` (one launch)."""
    _check("gradient_adjoint", gx, gy)
    gx, gy = gx.contiguous(), gy.contiguous()
    B, nx, ny = _geo(gx)
    out = torch.empty_like(gx)
    check(lib.bpk_ns_gradient_adjoint_f32(gx.data_ptr(), gy.data_ptr(), out.data_ptr(), B, nx,
                                          ny, float(dx), stream_ptr(gx.device)),
          "ns_step.gradient_adjoint")
    return out


class _StencilGradient(torch.autograd.Function):
    """(fx, fy) = ns_step stencil gradient of a [B, 1, H, W] field, differentiable to any
    order (the stencil is linear; its backward is the adjoint kernel, whose own backward
    is the stencil again)."""

    @staticmethod
    def forward(ctx, f, dx):
        ctx.dx = dx
        return gradient(f, dx)

    @staticmethod
    def backward(ctx, gx, gy):
        if gx is None:
            gx = torch.zeros_like(gy)
        if gy is None:
            gy = torch.zeros_like(gx)
        return _StencilGradientAdjoint.apply(gx, gy, ctx.dx), None


class _StencilGradientAdjoint(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gx, gy, dx):
        ctx.dx = dx
        return gradient_adjoint(gx, gy, dx)

    @staticmethod
    def backward(ctx, g):
        fx, fy = _StencilGradient.apply(g, ctx.dx)
        return fx, fy, None


def stencil_gradient(field, dx):
    """Differentiable (d/dx, d/dy) of a [B, 1, H, W] field on the ns_step stencil."""
    return _StencilGradient.apply(field, dx)
