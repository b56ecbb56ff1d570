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
