"""The PINN nets' spatial embedding on csrc/pinn_emb.hip (reference models/layers.py:517-521).

    f(x, y) = (sin(w * sqrt(x^2 + y^2)) + sin(w * sqrt((x.max() - x)^2 + (y.max() - y)^2))) / s

with x.max() / y.max() taken per copy when the batch holds k stacked copies of one batch
(models.layers.spatial_groups).  The PINN residual differentiates the nets w.r.t. x and y with
create_graph, then again (second derivatives), then the loss w.r.t. the parameters: as aten
ops the chain above costs ~15 launches forward and dozens per derivative pass.  Here:

    spatial_embedding -> _SpatialEmb        (forward: 2 launches, bit-identical values)
    its backward      -> _SpatialEmbVJP     (first derivatives incl. the max's evenly shared
                                             gradient: 2 launches, recorded under create_graph)
    that backward     -> bpk_spatial_emb_vjp2 (second derivatives: 2 launches)

Third derivatives are not provided (the residual never needs them: its second derivatives are
taken without create_graph).
"""
from __future__ import annotations

import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from ._lib import check, lib, mark_inputs, stream_ptr, want_grad

_WS: dict = {}


def _ws(n, k, device):
    """per-(device, copies) workspace for the per-copy partial sums; on the stream order of the
    caller (every launch that uses it is ordered on one stream, so reuse is safe)"""
    nbytes = int(lib.bpk_spatial_emb_workspace_bytes(n, k))
    key = (str(device), k)
    buf = _WS.get(key)
    if buf is None or buf.numel() * 4 < nbytes:
        buf = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=device)
        _WS[key] = buf
    return buf


def supported(x, y, k=1) -> bool:
    return (x.is_cuda and y.is_cuda and x.dtype == torch.float32 and y.dtype == torch.float32
            and x.shape == y.shape and bool(lib.bpk_spatial_emb_supported(x.numel(), int(k))))


def _vjp2(g, x, y, mxy, hx, hy, k, omega, s, want=(True, True, True)):
    n = x.numel()
    dg = torch.empty_like(x) if want[0] else None
    dx = torch.empty_like(x) if want[1] else None
    dy = torch.empty_like(x) if want[2] else None
    hx = None if hx is None else hx.contiguous()
    hy = None if hy is None else hy.contiguous()
    check(lib.bpk_spatial_emb_vjp2_f32(
        x.data_ptr(), y.data_ptr(), mxy.data_ptr(), g.data_ptr(),
        None if hx is None else hx.data_ptr(), None if hy is None else hy.data_ptr(),
        None if dg is None else dg.data_ptr(), None if dx is None else dx.data_ptr(),
        None if dy is None else dy.data_ptr(), _ws(n, k, x.device).data_ptr(), n, k, omega, s,
        stream_ptr(x.device)), "spatial_emb_vjp2")
    return dg, dx, dy


class _SpatialEmbVJP(Function):
    """(gx, gy) = the gradient of sum(g * f(x, y)) w.r.t. x and y (the max's term included)."""

    @staticmethod
    def forward(ctx, g, x, y, mxy, k, omega, s):
        mark_inputs(ctx, g, x, y, mxy, k, omega, s)
        g = g.contiguous()
        gx, gy = torch.empty_like(x), torch.empty_like(x)
        n = x.numel()
        check(lib.bpk_spatial_emb_vjp_f32(x.data_ptr(), y.data_ptr(), mxy.data_ptr(), g.data_ptr(),
                                          gx.data_ptr(), gy.data_ptr(), _ws(n, k, x.device).data_ptr(),
                                          n, k, omega, s, stream_ptr(x.device)), "spatial_emb_vjp")
        ctx.save_for_backward(g, x, y, mxy)
        ctx.k, ctx.omega, ctx.s = k, omega, s
        return gx, gy

    @staticmethod
    @once_differentiable
    def backward(ctx, hx, hy):
        g, x, y, mxy = ctx.saved_tensors
        want = (want_grad(ctx, 0), want_grad(ctx, 1), want_grad(ctx, 2))
        if not any(want) or (hx is None and hy is None):
            return (None,) * 7
        dg, dx, dy = _vjp2(g, x, y, mxy, hx, hy, ctx.k, ctx.omega, ctx.s, want)
        return dg, dx, dy, None, None, None, None


class _SpatialEmb(Function):
    @staticmethod
    def forward(ctx, x, y, k, omega, s):
        mark_inputs(ctx, x, y, k, omega, s)
        x, y = x.contiguous(), y.contiguous()
        out = torch.empty_like(x)
        mxy = torch.empty(k, 2, dtype=torch.float32, device=x.device)
        n = x.numel()
        check(lib.bpk_spatial_emb_fwd_f32(x.data_ptr(), y.data_ptr(), out.data_ptr(), mxy.data_ptr(),
                                          _ws(n, k, x.device).data_ptr(), n, k, omega, s,
                                          stream_ptr(x.device)), "spatial_emb")
        ctx.save_for_backward(x, y, mxy)
        ctx.k, ctx.omega, ctx.s = k, omega, s
        return out

    @staticmethod
    def backward(ctx, g):
        x, y, mxy = ctx.saved_tensors
        gx, gy = _SpatialEmbVJP.apply(g, x, y, mxy, ctx.k, ctx.omega, ctx.s)
        return (gx if want_grad(ctx, 0) else None, gy if want_grad(ctx, 1) else None,
                None, None, None)


def spatial_embedding(x, y, omega, s=1.0, k=1):
    """get_spatial_embedding(x, y, omega, s) on the native kernels; x.max() / y.max() per copy
    of a batch of k stacked copies.  Differentiable twice (create_graph on the first order)."""
    # contiguous outside the Function: it saves its inputs for the double backward
    return _SpatialEmb.apply(x.contiguous(), y.contiguous(), int(k), float(omega), float(s))
