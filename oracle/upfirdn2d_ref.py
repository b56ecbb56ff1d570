"""ORACLE (test infrastructure only) -- upfirdn2d restated on CPU.

Follows `upfirdn2d_native` (reference op/upfirdn2d.py:159-200): zero-insert
upsample, pad (negative = crop), convolve with the 180-degree-rotated kernel,
keep every `down`-th sample.  Two forms:
  * `upfirdn2d_np`   : numpy tap loop (any dtype), the independent checker;
  * `upfirdn2d_torch`: torch-CPU conv2d form (fast; used by nets_ref);
  * `upfirdn2d_native_seq`: the reference's own CPU op sequence, step for step (pad-based zero
    insertion, crop, 1-channel F.conv2d at full resolution, then the `[::down]` slice) -- the
    upfirdn2d CPU baseline of bench.py times this one.
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


def upfirdn2d_native_seq(x, k, up=1, down=1, pad=(0, 0)):
    """The reference CPU path's op sequence (op/upfirdn2d.py:159-200, `upfirdn2d_native` with
    the symmetric (up, down, pad) of `upfirdn2d`, op/upfirdn2d.py:145-156): the view/pad zero
    insertion, the pad + crop, one single-channel conv2d over every plane at the upsampled
    resolution, and the stride taken afterwards by slicing (so a down-2 op convolves 4x the
    output pixels, as the reference does)."""
    _, channel, in_h, in_w = x.shape
    kh, kw = k.shape
    p0, p1 = pad
    out = x.reshape(-1, in_h, 1, in_w, 1, 1)
    out = F.pad(out, [0, 0, 0, up - 1, 0, 0, 0, up - 1])
    out = out.view(-1, in_h * up, in_w * up, 1)
    out = F.pad(out, [0, 0, max(p0, 0), max(p1, 0), max(p0, 0), max(p1, 0)])
    out = out[:, max(-p0, 0):out.shape[1] - max(-p1, 0), max(-p0, 0):out.shape[2] - max(-p1, 0), :]
    out = out.permute(0, 3, 1, 2).reshape(-1, 1, in_h * up + p0 + p1, in_w * up + p0 + p1)
    w = torch.flip(k, [0, 1]).view(1, 1, kh, kw).to(x.dtype)
    out = F.conv2d(out, w)
    out = out.reshape(-1, 1, in_h * up + p0 + p1 - kh + 1, in_w * up + p0 + p1 - kw + 1)
    out = out.permute(0, 2, 3, 1)[:, ::down, ::down, :]
    oh = (in_h * up + p0 + p1 - kh) // down + 1
    ow = (in_w * up + p0 + p1 - kw) // down + 1
    return out.reshape(-1, channel, oh, ow)
