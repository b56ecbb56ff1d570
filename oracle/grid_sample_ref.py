"""ORACLE (test infrastructure only) -- bilinear grid_sample fwd / bwd / grad2 on CPU.

fwd / bwd are ATen's CPU kernels (the reference calls ATen for these,
op/grid_sample.py:39-60).  grad2 restates the reference's double-backward kernel
(op/grid_sample_kernel.cu:27-210) with vectorised torch ops; it is pinned by
float64 finite differences of the first backward (tests/test_oracle_grid_sample.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

_PM = {0: "zeros", 1: "border"}


def fwd(inp, grid, padding_mode=0, align_corners=True):
    return F.grid_sample(inp, grid, mode="bilinear", padding_mode=_PM[padding_mode],
                         align_corners=align_corners)


def bwd(gout, inp, grid, padding_mode=0, align_corners=True):
    op = torch.ops.aten.grid_sampler_2d_backward
    return op(gout, inp, grid, 0, padding_mode, align_corners, [True, True])


def _source_index(coord, size, padding_mode, align):
    if align:
        mult = (size - 1) / 2
        ix = (coord + 1) / 2 * (size - 1)
    else:
        mult = size / 2
        ix = ((coord + 1) * size - 1) / 2
    gmult = torch.full_like(coord, mult)
    if padding_mode == 1:
        lo = ix <= 0
        hi = ix >= size - 1
        gmult = torch.where(lo | hi, torch.zeros_like(gmult), gmult)
        ix = torch.where(lo, torch.zeros_like(ix), torch.where(hi, torch.full_like(ix, size - 1), ix))
    return ix, gmult


def grad2(g2_inp, g2_grid, gout, inp, grid, padding_mode=0, align_corners=True):
    """Returns (grad_grad_output, grad_input, grad_grid) like gridsample_grad2.grad2_2d."""
    N, C, H, W = inp.shape
    Ho, Wo = grid.shape[1:3]
    ix, gxm = _source_index(grid[..., 0], W, padding_mode, align_corners)
    iy, gym = _source_index(grid[..., 1], H, padding_mode, align_corners)
    x0 = torch.floor(ix)
    y0 = torch.floor(iy)
    x1, y1 = x0 + 1, y0 + 1
    nw = (x1 - ix) * (y1 - iy)
    ne = (ix - x0) * (y1 - iy)
    sw = (x1 - ix) * (iy - y0)
    se = (ix - x0) * (iy - y0)
    dx = g2_grid[..., 0] * gxm
    dy = g2_grid[..., 1] * gym
    nw_t = -dx * (y1 - iy) - dy * (x1 - ix)
    ne_t = dx * (y1 - iy) - dy * (ix - x0)
    sw_t = -dx * (iy - y0) + dy * (x1 - ix)
    se_t = dx * (iy - y0) + dy * (ix - x0)

    def gather(src, yy, xx):
        ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
        yi = yy.clamp(0, H - 1).long()
        xi = xx.clamp(0, W - 1).long()
        flat = (yi * W + xi).reshape(N, 1, Ho * Wo).expand(N, C, Ho * Wo)
        v = torch.gather(src.reshape(N, C, H * W), 2, flat).reshape(N, C, Ho, Wo)
        return v * ok[:, None].to(v.dtype), ok, flat

    corners = [(y0, x0, nw, nw_t), (y0, x1, ne, ne_t), (y1, x0, sw, sw_t), (y1, x1, se, se_t)]
    ggo = torch.zeros_like(gout)
    gin = torch.zeros_like(inp).reshape(N, C, H * W)
    vals = []
    for yy, xx, w, tmp in corners:
        v, ok, flat = gather(inp, yy, xx)
        g2v, _, _ = gather(g2_inp, yy, xx)
        vals.append((v, g2v))
        ggo = ggo + g2v * w[:, None] + v * tmp[:, None]
        contrib = (tmp[:, None] * gout) * ok[:, None].to(inp.dtype)
        gin.scatter_add_(2, flat, contrib.reshape(N, C, Ho * Wo))
    (nwv, g2nw), (nev, g2ne), (swv, g2sw), (sev, g2se) = vals
    dxy = nwv - nev - swv + sev
    gix = gout * (-g2nw * (y1 - iy)[:, None] + g2ne * (y1 - iy)[:, None]
                  - g2sw * (iy - y0)[:, None] + g2se * (iy - y0)[:, None]) + gout * dy[:, None] * dxy
    giy = gout * (-g2nw * (x1 - ix)[:, None] - g2ne * (ix - x0)[:, None]
                  + g2sw * (x1 - ix)[:, None] + g2se * (ix - x0)[:, None]) + gout * dx[:, None] * dxy
    ggrid = torch.stack([gix.sum(1) * gxm, giy.sum(1) * gym], dim=-1)
    return ggo, gin.reshape(N, C, H, W), ggrid


# ---------------------------------------------------------------- 3-D (trilinear)

def fwd3(inp, grid, padding_mode=0, align_corners=True):
    return F.grid_sample(inp, grid, mode="bilinear", padding_mode=_PM[padding_mode],
                         align_corners=align_corners)


def bwd3(gout, inp, grid, padding_mode=0, align_corners=True):
    op = torch.ops.aten.grid_sampler_3d_backward
    return op(gout, inp, grid, 0, padding_mode, align_corners, [True, True])


def grad3(g2_inp, g2_grid, gout, inp, grid, padding_mode=0, align_corners=True):
    """(grad_grad_output, grad_input, grad_grid) like gridsample_grad2.grad2_3d: the
    reference's op/grid_sample_kernel.cu:212-533 with vectorised torch ops, written per
    corner (bz, by, bx) as the reference's tnw .. bse terms: weight Wx Wy Wz, its
    derivative along an axis replaces that axis' factor by -1 (corner 0) / +1 (corner 1)."""
    N, C, D, H, W = inp.shape
    Do, Ho, Wo = grid.shape[1:4]
    S = Do * Ho * Wo
    ix, gxm = _source_index(grid[..., 0], W, padding_mode, align_corners)
    iy, gym = _source_index(grid[..., 1], H, padding_mode, align_corners)
    iz, gzm = _source_index(grid[..., 2], D, padding_mode, align_corners)
    x0, y0, z0 = torch.floor(ix), torch.floor(iy), torch.floor(iz)
    Wx = [(x0 + 1) - ix, ix - x0]
    Wy = [(y0 + 1) - iy, iy - y0]
    Wz = [(z0 + 1) - iz, iz - z0]
    dx = g2_grid[..., 0] * gxm
    dy = g2_grid[..., 1] * gym
    dz = g2_grid[..., 2] * gzm
    ggo = torch.zeros_like(gout)
    gin = torch.zeros_like(inp).reshape(N, C, D * H * W)
    dxy = torch.zeros_like(gout)
    dxz = torch.zeros_like(gout)
    dyz = torch.zeros_like(gout)
    ax = torch.zeros_like(gout)
    ay = torch.zeros_like(gout)
    az = torch.zeros_like(gout)
    e = lambda t: t[:, None]
    for bz in (0, 1):
        for by in (0, 1):
            for bx in (0, 1):
                sx, sy, sz = (1 if bx else -1), (1 if by else -1), (1 if bz else -1)
                zz, yy, xx = z0 + bz, y0 + by, x0 + bx
                ok = (zz >= 0) & (zz < D) & (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
                flat = ((zz.clamp(0, D - 1) * H + yy.clamp(0, H - 1)) * W + xx.clamp(0, W - 1)).long()
                flat = flat.reshape(N, 1, S).expand(N, C, S)
                okf = e(ok).to(inp.dtype)
                v = torch.gather(inp.reshape(N, C, -1), 2, flat).reshape(gout.shape) * okf
                g2 = torch.gather(g2_inp.reshape(N, C, -1), 2, flat).reshape(gout.shape) * okf
                w = Wx[bx] * Wy[by] * Wz[bz]
                tmp = sx * dx * Wy[by] * Wz[bz] + sy * dy * Wx[bx] * Wz[bz] + sz * dz * Wx[bx] * Wy[by]
                ggo = ggo + g2 * e(w) + v * e(tmp)
                gin.scatter_add_(2, flat, ((e(tmp) * gout) * okf).reshape(N, C, S))
                dxy = dxy + sx * sy * v * e(Wz[bz])
                dxz = dxz + sx * sz * v * e(Wy[by])
                dyz = dyz + sy * sz * v * e(Wx[bx])
                ax = ax + sx * g2 * e(Wy[by] * Wz[bz])
                ay = ay + sy * g2 * e(Wx[bx] * Wz[bz])
                az = az + sz * g2 * e(Wx[bx] * Wy[by])
    gix = (gout * ax + gout * (e(dz) * dxz + e(dy) * dxy)).sum(1) * gxm
    giy = (gout * ay + gout * (e(dx) * dxy + e(dz) * dyz)).sum(1) * gym
    giz = (gout * az + gout * (e(dx) * dxz + e(dy) * dyz)).sum(1) * gzm
    return ggo, gin.reshape(inp.shape), torch.stack([gix, giy, giz], dim=-1)
