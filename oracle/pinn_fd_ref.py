"""ORACLE (test infrastructure only) -- CPU restatements for the PINN / UKF paths that run
on the ns_step stencil:

  * `fd_residual_mse`: the stencil residual of `PINN.equation_mse_fd` (the north star's
    "PINN residual reusing the ns_step stencil"), in float64 with the C stencil oracle's
    derivatives (oracle/ns_step_ref.c ns_ref_gradient = reference diff_x / diff_y,
    op/ns_step_kernel.cu:50-75) and the residual formula of reference pinn.py:101-111;
  * `patch` / `unpatch` / `ns_dynamics`: reference pinn_kalman/ukf_utils.py:8-22, 95-119
    with explicit index loops / numpy reshapes (no torchvision), the three ns_step calls
    through the C oracle.
"""
from __future__ import annotations

import numpy as np

from oracle import ns_step_ref


def _grad64(f, h):
    """(d/dx, d/dy) with the stencil of the C oracle's ns_ref_gradient (central differences
    / 2h inside, one-sided / h at the borders; x = last axis, y = second to last), in
    float64; pinned against the C oracle by check_stencil_matches_c."""
    f = np.asarray(f, np.float64)
    gx = np.empty_like(f)
    gy = np.empty_like(f)
    gx[..., 1:-1] = (f[..., 2:] - f[..., :-2]) / (2 * h)
    gx[..., 0] = (f[..., 1] - f[..., 0]) / h
    gx[..., -1] = (f[..., -1] - f[..., -2]) / h
    gy[..., 1:-1, :] = (f[..., 2:, :] - f[..., :-2, :]) / (2 * h)
    gy[..., 0, :] = (f[..., 1, :] - f[..., 0, :]) / h
    gy[..., -1, :] = (f[..., -1, :] - f[..., -2, :]) / h
    return gx, gy


def check_stencil_matches_c(f, h):
    """The float64 stencil above equals the C oracle (float32) to rounding."""
    rx, ry = ns_step_ref.gradient(np.asarray(f, np.float32), h)
    gx, gy = _grad64(f, np.float32(h))
    return max(np.abs(gx - rx).max() / max(1.0, np.abs(rx).max()),
               np.abs(gy - ry).max() / max(1.0, np.abs(ry).max()))


def fd_residual_mse(u, v, p, u_t, v_t, h, Re):
    h = np.float64(np.float32(h))
    ux, uy = _grad64(u, h)
    vx, vy = _grad64(v, h)
    px, py = _grad64(p, h)
    uxx = _grad64(ux, h)[0]
    uyy = _grad64(uy, h)[1]
    vxx = _grad64(vx, h)[0]
    vyy = _grad64(vy, h)[1]
    u = np.asarray(u, np.float64)
    v = np.asarray(v, np.float64)
    ut = np.asarray(u_t, np.float64)[:, None, None, None]
    vt = np.asarray(v_t, np.float64)[:, None, None, None]
    nu = 1.0 / Re
    rx = ut + (u * ux + v * uy) + px - nu * (uxx + uyy)
    ry = vt + (u * vx + v * vy) + py - nu * (vxx + vyy)
    rm = ux + vy
    return float((rx ** 2).mean() + (ry ** 2).mean() + (rm ** 2).mean())


def patch(x, p):
    """[B, C, H, W] -> rows (c, b, i, j) of p*p values (reference ukf_utils.py:8-15)."""
    B, C, H, W = x.shape
    out = np.empty((C, B, H // p, W // p, p * p), x.dtype)
    for c in range(C):
        for b in range(B):
            for i in range(H // p):
                for j in range(W // p):
                    out[c, b, i, j] = x[b, c, i * p:(i + 1) * p, j * p:(j + 1) * p].reshape(-1)
    return out.reshape(-1, p * p)


def unpatch(rows, p, f, C):
    n = f // p
    r = rows.reshape(C, -1, n, n, p, p)
    B = r.shape[1]
    out = np.empty((B, C, f, f), rows.dtype)
    for c in range(C):
        for b in range(B):
            for i in range(n):
                for j in range(n):
                    out[b, c, i * p:(i + 1) * p, j * p:(j + 1) * p] = r[c, b, i, j]
    return out


def ns_dynamics(states, p, f):
    """NSDynamics.forward (reference ukf_utils.py:95-119): unpatch, the three ns_step ops
    (C oracle, compat quirk on as in the reference), patch; covariance 1e-8 I."""
    u = unpatch(states, p, f, 4)
    fd, v, pr = u[:, 0:1], u[:, 1:3], u[:, 3:4]
    dt, dx = 0.0005 * 5, 1 / 200
    v = ns_step_ref.update_velocity(v, pr, dt, dx, True)
    pr = ns_step_ref.update_pressure(pr, v, dt, dx)
    fd = ns_step_ref.update_density(fd, v, dt, dx)
    st = patch(np.concatenate([fd, v, pr], 1), p)
    return st, np.repeat(np.eye(p * p, dtype=np.float32)[None] * np.float32(1e-8), st.shape[0], 0)
