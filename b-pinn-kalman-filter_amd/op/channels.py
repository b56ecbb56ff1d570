"""Concatenation and channel swap with derivatives of every order that stay single ops.

The PINN residual (reference pinn.py:72-111) differentiates FlowNet / PressureNet three
times (the first-order sensitivities w.r.t. x, y, t with create_graph, the second-order ones,
then the loss w.r.t. the parameters).  torch.cat's backward returns narrow views of the
gradient; differentiated again, every view becomes `slice_backward` -- a zero fill of the
whole gradient plus a copy into the slice -- and the pieces are summed with adds: 3k - 1
launches per k-input concatenation per pass, ~2.5 k of the PINN step's launches.  Here the
backward of `cat` is `split` (views, no launch) and the backward of `split` is one `cat`.
The reference's own ops (models/flownet.py: torch.cat in SubpixelRefinement, Upsample,
PressureNet; layers.py get_timestep_embedding) keep their values bit for bit: the forward is
torch.cat itself.
"""
from __future__ import annotations

import torch
from torch.autograd import Function

from ._lib import check, lib, stream_ptr


class _Cat(Function):
    @staticmethod
    def forward(ctx, dim, *xs):
        ctx.dim = dim
        ctx.sizes = tuple(x.shape[dim] for x in xs)
        return torch.cat(xs, dim)

    @staticmethod
    def backward(ctx, g):
        return (None,) + tuple(_Split.apply(g, ctx.dim, ctx.sizes))


class _Split(Function):
    @staticmethod
    def forward(ctx, g, dim, sizes):
        ctx.dim = dim
        ctx.shape = tuple(g.shape)
        ctx.sizes = sizes
        ctx.set_materialize_grads(False)
        return tuple(torch.split(g, list(sizes), dim))

    @staticmethod
    def backward(ctx, *gs):
        if all(g is not None for g in gs):
            return _Cat.apply(ctx.dim, *gs), None, None
        # pieces nobody used (PINN.forward_residual_copies reads copy 0 of most splits): one
        # zero fill and a copy per used piece, not a fill per unused piece plus a cat
        present = tuple(g is not None for g in gs)
        return _PadCat.apply(ctx.dim, ctx.sizes, present, ctx.shape,
                             *[g for g in gs if g is not None]), None, None


class _PadCat(Function):
    """cat along `dim` of the pieces marked present, zeros for the others; backward: views of
    the present pieces (a split)."""

    @staticmethod
    def forward(ctx, dim, sizes, present, shape, *gs):
        ctx.dim, ctx.sizes, ctx.present = dim, sizes, present
        out = gs[0].new_zeros(shape) if gs else torch.zeros(shape)
        it = iter(gs)
        off = 0
        for sz, p in zip(sizes, present):
            if p:
                out.narrow(dim, off, sz).copy_(next(it))
            off += sz
        return out

    @staticmethod
    def backward(ctx, gout):
        pieces = _Split.apply(gout, ctx.dim, ctx.sizes)
        return (None, None, None, None) + tuple(
            q for q, p in zip(pieces, ctx.present) if p)


def cat(tensors, dim=0):
    """torch.cat(tensors, dim) whose derivatives of every order are single cat / split ops."""
    tensors = list(tensors)
    if len(tensors) == 1:
        return tensors[0]
    if not torch.is_grad_enabled() or not any(t.requires_grad for t in tensors):
        return torch.cat(tensors, dim)
    return _Cat.apply(dim % tensors[0].dim(), *tensors)


def split(x, sizes, dim=0):
    """torch.split(x, sizes, dim) whose backward is one cat (and that cat's backward a split)."""
    sizes = tuple(int(v) for v in sizes)
    if not torch.is_grad_enabled() or not x.requires_grad:
        return tuple(torch.split(x, list(sizes), dim))
    return _Split.apply(x, dim % x.dim(), sizes)


class _SwapScale(Function):
    """out[:, 0] = u[:, 1] / c0, out[:, 1] = u[:, 0] / c1 for u [B, 2, ...]: a linear map whose
    adjoint is the same map with the divisors exchanged."""

    @staticmethod
    def forward(ctx, u, c0, c1):
        ctx.c = (c0, c1)
        if u.is_cuda and u.dtype == torch.float32:
            # one launch (csrc/channels.hip) instead of two divisions into output slices; the
            # gradients coming back through project's NHWC grid view are channels-last and run
            # in that layout (no copy)
            cl = u.dim() == 4 and not u.is_contiguous() and u.permute(0, 2, 3, 1).is_contiguous()
            if not cl:
                u = u.contiguous()
            out = torch.empty_like(u)  # same strides as u (dense)
            if out.stride() != u.stride():
                raise RuntimeError(f"swap_scale: output strides {out.stride()} != {u.stride()}")
            check(lib.bpk_swap_scale_f32(u.data_ptr(), out.data_ptr(), u.shape[0],
                                         u[0, 0].numel(), c0, c1, int(cl), stream_ptr(u.device)),
                  "swap_scale")
            return out
        out = torch.empty_like(u)  # float64 (gradcheck) / CPU tensors
        torch.div(u[:, 1:2], c0, out=out[:, 0:1])
        torch.div(u[:, 0:1], c1, out=out[:, 1:2])
        return out

    @staticmethod
    def backward(ctx, g):
        c0, c1 = ctx.c
        return _SwapScale.apply(g, c1, c0), None, None


def swap_scale(u, c0, c1):
    """torch.cat([u[:, 1:2] / c0, u[:, 0:1] / c1], 1), every derivative one such op."""
    if u.shape[1] != 2:
        raise RuntimeError(f"swap_scale: 2 channels expected, got {tuple(u.shape)}")
    if not torch.is_grad_enabled() or not u.requires_grad:
        return torch.cat([u[:, 1:2] / c0, u[:, 0:1] / c1], 1)
    return _SwapScale.apply(u, float(c0), float(c1))
