"""ORACLE (test infrastructure only) -- upfirdn2d restated on CPU.

Follows `upfirdn2d_native` (reference op/upfirdn2d.py:159-200): zero-insert
upsample, pad (negative = crop), convolve with the 180-degree-rotated kernel,
keep every `down`-th sample.  Two forms:
  * `upfirdn2d_np`   : numpy tap loop (any dtype), the independent checker;
  * `upfirdn2d_torch`: torch-CPU conv2d form (fast; used by nets_ref / cpu baseline).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def out_size(in_h, in_w, kh, kw, up, down, pad):
    ux, uy = up
    dx, dy = down
    px0, px1, py0, py1 = pad
    return (in_h * uy + py0 + py1 - kh) // dy + 1, (in_w * ux + px0 + px1 - kw) // dx + 1


def upfirdn2d_np(x, k, up=(1, 1), down=(1, 1), pad=(0, 0, 0, 0)):
    """x [..., H, W] numpy; returns [..., out_h, out_w] in x.dtype (accumulates in float64)."""
    x = np.asarray(x)
    k = np.asarray(k, dtype=np.float64)
    ux, uy = up
    dx, dy = down
    px0, px1, py0, py1 = pad
    H, W = x.shape[-2:]
    kh, kw = k.shape
    oh, ow = out_size(H, W, kh, kw, up, down, pad)
    Uh, Uw = H * uy, W * ux
    # zero-inserted image U placed at offset M inside a zero canvas Z; the padded image of
    # the reference is P[r, c] = U[r - py0, c - px0] = Z[r - py0 + M, c - px0 + M]
    M = max(abs(px0), abs(px1), abs(py0), abs(py1), kh, kw) + 1
    Z = np.zeros(x.shape[:-2] + (Uh + 2 * M, Uw + 2 * M), dtype=np.float64)
    Z[..., M:M + Uh:uy, M:M + Uw:ux] = x
    out = np.zeros(x.shape[:-2] + (oh, ow), dtype=np.float64)
    for i in range(kh):
        for j in range(kw):
            w = k[kh - 1 - i, kw - 1 - j]
            ys, xs = i - py0 + M, j - px0 + M
            out += w * Z[..., ys:ys + (oh - 1) * dy + 1:dy, xs:xs + (ow - 1) * dx + 1:dx]
    return out.astype(x.dtype)


def upfirdn2d_torch(x, k, up=1, down=1, pad=(0, 0)):
    """Same op with torch CPU ops, symmetric (up, down, pad) on both axes (op/upfirdn2d.py:145)."""
    N, C, H, W = x.shape
    kh, kw = k.shape
    p0, p1 = pad
    if up > 1:
        U = x.new_zeros((N, C, H * up, W * up))
        U[:, :, ::up, ::up] = x
    else:
        U = x
    U = F.pad(U, (max(p0, 0), max(p1, 0), max(p0, 0), max(p1, 0)))
    if p0 < 0 or p1 < 0:
        U = U[:, :, max(-p0, 0):U.shape[2] - max(-p1, 0), max(-p0, 0):U.shape[3] - max(-p1, 0)]
    w = torch.flip(k, [0, 1]).to(x.dtype).reshape(1, 1, kh, kw)
    out = F.conv2d(U.reshape(N * C, 1, U.shape[2], U.shape[3]), w, stride=down)
    return out.reshape(N, C, out.shape[2], out.shape[3])
