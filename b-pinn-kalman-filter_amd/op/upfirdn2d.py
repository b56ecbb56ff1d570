"""`op.upfirdn2d` on the gfx950 HIP kernel (csrc/upfirdn2d.hip).

Public signature kept from the reference: `upfirdn2d(input[N,C,H,W], kernel[kh,kw],
up=1, down=1, pad=(p0, p1))` with `pad` applied to both axes
(op/upfirdn2d.py:145-156).  Differentiable to any order: the backward of the op
is the same op with up <-> down, the 180-degree-rotated kernel and the adjoint
padding of op/upfirdn2d.py:111-116; the backward of the backward is the forward
again (op/upfirdn2d.py:64-85).

Unlike the reference there is no CPU branch (`upfirdn2d_native`): a CPU tensor is
an error, so a GPU run can never silently fall back to the host.
"""
from __future__ import annotations

import torch
from torch.autograd import Function

from ._lib import check, lib, require_hip, stream_ptr


def _out_size(in_h, in_w, kh, kw, up, down, pad):
    up_x, up_y = up
    down_x, down_y = down
    px0, px1, py0, py1 = pad
    out_h = (in_h * up_y + py0 + py1 - kh) // down_y + 1
    out_w = (in_w * up_x + px0 + px1 - kw) // down_x + 1
    return out_h, out_w


def upfirdn2d_raw(x: torch.Tensor, kernel: torch.Tensor, up=(1, 1), down=(1, 1),
                  pad=(0, 0, 0, 0)) -> torch.Tensor:
    """One launch on [N, C, H, W] (minor = 1) or [major, H, W, minor] via `minor`."""
    require_hip(x, kernel, what="upfirdn2d")
    if x.dtype not in (torch.float32, torch.float64):
        raise RuntimeError(f"upfirdn2d: unsupported dtype {x.dtype}")
    x = x.contiguous()
    kernel = kernel.to(device=x.device, dtype=x.dtype).contiguous()
    n, c, in_h, in_w = x.shape
    kh, kw = kernel.shape
    out_h, out_w = _out_size(in_h, in_w, kh, kw, up, down, pad)
    if out_h <= 0 or out_w <= 0:
        raise RuntimeError(f"upfirdn2d: empty output {out_h}x{out_w}")
    out = torch.empty((n, c, out_h, out_w), device=x.device, dtype=x.dtype)
    fn = lib.bpk_upfirdn2d_f32 if x.dtype == torch.float32 else lib.bpk_upfirdn2d_f64
    check(fn(x.data_ptr(), kernel.data_ptr(), out.data_ptr(), n * c, in_h, in_w, 1, kh, kw,
             up[0], up[1], down[0], down[1], pad[0], pad[1], pad[2], pad[3], out_h, out_w,
             stream_ptr(x.device)), "upfirdn2d")
    return out


def _adjoint_pad(in_h, in_w, kh, kw, up, down, pad, out_h, out_w):
    up_x, up_y = up
    down_x, down_y = down
    px0, px1, py0, py1 = pad
    gpx0 = kw - px0 - 1
    gpy0 = kh - py0 - 1
    gpx1 = in_w * up_x - out_w * down_x + px0 - up_x + 1
    gpy1 = in_h * up_y - out_h * down_y + py0 - up_y + 1
    return gpx0, gpx1, gpy0, gpy1


class _UpFirDn2dGrad(Function):
    """d(upfirdn2d)/d(input) applied to grad_output; its own derivative is the forward op."""

    @staticmethod
    def forward(ctx, grad_out, kernel, up, down, pad, in_size):
        in_h, in_w = in_size
        kh, kw = kernel.shape
        out_h, out_w = grad_out.shape[-2:]
        gpad = _adjoint_pad(in_h, in_w, kh, kw, up, down, pad, out_h, out_w)
        grad_in = upfirdn2d_raw(grad_out, torch.flip(kernel, [0, 1]), up=down, down=up, pad=gpad)
        ctx.save_for_backward(kernel)
        ctx.up, ctx.down, ctx.pad = up, down, pad
        return grad_in

    @staticmethod
    def backward(ctx, gg_in):
        kernel, = ctx.saved_tensors
        gg_out = _UpFirDn2dFn.apply(gg_in, kernel, ctx.up, ctx.down, ctx.pad)
        return gg_out, None, None, None, None, None


class _UpFirDn2dFn(Function):
    @staticmethod
    def forward(ctx, x, kernel, up, down, pad):
        ctx.save_for_backward(kernel)
        ctx.up, ctx.down, ctx.pad = up, down, pad
        ctx.in_size = tuple(x.shape[-2:])
        return upfirdn2d_raw(x, kernel, up, down, pad)

    @staticmethod
    def backward(ctx, grad_out):
        kernel, = ctx.saved_tensors
        grad_in = _UpFirDn2dGrad.apply(grad_out.contiguous(), kernel, ctx.up, ctx.down, ctx.pad,
                                       ctx.in_size)
        return grad_in, None, None, None, None


def upfirdn2d(input, kernel, up=1, down=1, pad=(0, 0)):
    """Reference API (op/upfirdn2d.py:145-156): same (up, down, pad) on both axes."""
    require_hip(input, what="upfirdn2d")
    if not torch.is_tensor(kernel):
        kernel = torch.as_tensor(kernel, dtype=input.dtype, device=input.device)
    return _UpFirDn2dFn.apply(input, kernel, (up, up), (down, down),
                              (pad[0], pad[1], pad[0], pad[1]))


def upfirdn2d_xy(input, kernel, up=(1, 1), down=(1, 1), pad=(0, 0, 0, 0)):
    """Per-axis variant mirroring the extension signature (op/upfirdn2d.cpp:12-22)."""
    require_hip(input, what="upfirdn2d")
    return _UpFirDn2dFn.apply(input, kernel, tuple(up), tuple(down), tuple(pad))
