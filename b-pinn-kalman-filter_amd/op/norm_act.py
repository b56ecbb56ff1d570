"""Fused GroupNorm(+bias)(+SiLU) and the skip-rescale residual, with autograd.

These are the build's fusions of the NCSN++/DDPM++ block arithmetic
(models/layerspp.py:242-274 and :200-209):
  * `group_norm_act(x, gn, act, bias_nc)`  = act(GroupNorm(x + bias_nc[:, :, None, None]))
    -- one HIP launch (csrc/group_norm.hip) instead of add + group_norm + silu;
  * `residual_rescale(x, h, bias, div)`    = (x + (h + bias[c])) / div
    -- folds Conv_1's bias and the skip connection into one pass;
  * `instance_norm_act(x)` = ELU(InstanceNorm2d(x)) of PressureNet's ResidualBlock
    (models/layers.py:438-491), forward / backward / double backward one kernel each.
"""
from __future__ import annotations

import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from ._lib import check, lib, require_hip, stream_ptr, mark_inputs, want_grad

ACT_NONE, ACT_SILU = 0, 1


def _ws(N, C, HW, G, device):
    nb = lib.bpk_group_norm_workspace_bytes(N, C, HW, G)
    return torch.empty(max(nb // 4, 1), device=device, dtype=torch.float32) if nb > 0 else None


class _GroupNormAct(Function):
    @staticmethod
    def forward(ctx, x, bias_nc, weight, bias, num_groups, eps, act):
        mark_inputs(ctx, x, bias_nc, weight, bias)
        require_hip(x, what="group_norm_act")
        if x.dtype != torch.float32:
            raise RuntimeError(f"group_norm_act: float32 required, got {x.dtype}")
        x = x.contiguous()
        N, C = x.shape[:2]
        HW = x.numel() // max(N * C, 1)
        y = torch.empty_like(x)
        mean = torch.empty((N, num_groups), device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        bnc = bias_nc.contiguous() if bias_nc is not None else None
        ws = _ws(N, C, HW, num_groups, x.device)
        check(lib.bpk_group_norm_fwd_f32(
            x.data_ptr(), bnc.data_ptr() if bnc is not None else None,
            weight.data_ptr() if weight is not None else None,
            bias.data_ptr() if bias is not None else None, y.data_ptr(), mean.data_ptr(),
            rstd.data_ptr(), ws.data_ptr() if ws is not None else None, N, C, HW, num_groups,
            float(eps), act, stream_ptr(x.device)), "group_norm_act")
        ctx.save_for_backward(x, bnc, weight, bias, mean, rstd)
        ctx.num_groups, ctx.act = num_groups, act
        ctx.has_bnc = bnc is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, bnc, weight, bias, mean, rstd = ctx.saved_tensors
        dx, d_bnc, dw, dbeta = group_norm_act_backward(
            dy, x, bnc, weight, bias, mean, rstd, ctx.num_groups, ctx.act,
            ctx.has_bnc and want_grad(ctx, 1), want_grad(ctx, 2), want_grad(ctx, 3))
        return dx, d_bnc, dw, dbeta, None, None, None


def group_norm_act_backward(dy, x, bnc, weight, bias, mean, rstd, G, act, want_bnc, want_w,
                            want_b, addend=None):
    """(dx, d bias_nc, d gamma, d beta) of y = act(GroupNorm(x + bias_nc)) for the output
    gradient dy, from the forward's group statistics (None where not wanted).  `addend`: another
    consumer's gradient of x, added into dx by the same kernel (d bias_nc stays the GroupNorm
    part alone)."""
    dy = dy.contiguous()
    N, C = x.shape[:2]
    HW = x.numel() // max(N * C, 1)
    dx = torch.empty_like(x)
    need_affine = weight is not None and (want_w or want_b)
    dg = torch.empty((N, C), device=x.device, dtype=torch.float32) if need_affine else None
    db = torch.empty((N, C), device=x.device, dtype=torch.float32) if need_affine else None
    ws = _ws(N, C, HW, G, x.device)
    late = None  # d bias_nc sums the GroupNorm part of dx: with it, the addend comes after
    if addend is not None:
        addend = addend.contiguous()
        if addend.shape != x.shape or addend.dtype != x.dtype:
            raise RuntimeError(f"group_norm_act_backward: addend {tuple(addend.shape)} vs x "
                               f"{tuple(x.shape)}")
        if bnc is not None and want_bnc:
            late, addend = addend, None
    check(lib.bpk_group_norm_bwd_add_f32(
        dy.data_ptr(), x.data_ptr(), bnc.data_ptr() if bnc is not None else None,
        weight.data_ptr() if weight is not None else None,
        bias.data_ptr() if bias is not None else None, mean.data_ptr(), rstd.data_ptr(),
        addend.data_ptr() if addend is not None else None,
        dx.data_ptr(), dg.data_ptr() if dg is not None else None,
        db.data_ptr() if db is not None else None, ws.data_ptr() if ws is not None else None,
        N, C, HW, G, act, stream_ptr(x.device)), "group_norm_act_bwd")
    # the three reductions in one launch (bpk_group_norm_param_grads_f32)
    d_bnc = (torch.empty((N, C), device=x.device, dtype=torch.float32)
             if (bnc is not None and want_bnc) else None)
    dw = torch.empty(C, device=x.device, dtype=torch.float32) if dg is not None and want_w else None
    dbeta = (torch.empty(C, device=x.device, dtype=torch.float32)
             if db is not None and want_b else None)
    if d_bnc is not None or dw is not None or dbeta is not None:
        check(lib.bpk_group_norm_param_grads_f32(
            dx.data_ptr(), dg.data_ptr() if dg is not None else None,
            db.data_ptr() if db is not None else None,
            d_bnc.data_ptr() if d_bnc is not None else None,
            dw.data_ptr() if dw is not None else None,
            dbeta.data_ptr() if dbeta is not None else None, N, C, HW, stream_ptr(x.device)),
            "group_norm_param_grads")
    if late is not None:
        dx = late + dx
    return dx, d_bnc, dw, dbeta


class _GroupNormActFanout(Function):
    """(act(GroupNorm(x)), x): a residual block's input feeds its first GroupNorm and its skip
    (identity, 1x1 projection or resampling).  Both gradients reach this one node and the
    skip's is added inside the GroupNorm backward kernel (bpk_group_norm_bwd_add_f32's addend)
    instead of by an autograd accumulation launch over the block's input.  First order (the
    training backward)."""

    @staticmethod
    def forward(ctx, x, weight, bias, num_groups, eps, act):
        ctx.set_materialize_grads(False)
        y = _GroupNormAct.forward(ctx, x, None, weight, bias, num_groups, eps, act)
        mark_inputs(ctx, x, weight, bias, num_groups, eps, act)  # this Function's positions
        return y, x.view_as(x)

    @staticmethod
    @once_differentiable
    def backward(ctx, dy, dskip):
        x, bnc, weight, bias, mean, rstd = ctx.saved_tensors
        if dy is None:
            return dskip, None, None, None, None, None
        dx, _, dw, dbeta = group_norm_act_backward(
            dy, x, None, weight, bias, mean, rstd, ctx.num_groups, ctx.act, False,
            weight is not None and want_grad(ctx, 1), bias is not None and want_grad(ctx, 2),
            addend=dskip)
        return dx, dw, dbeta, None, None, None


def group_norm_act_fanout(x, gn: torch.nn.GroupNorm, act: int = ACT_SILU):
    """(act(GroupNorm(x)), x) with the skip's gradient joining the norm's inside the backward
    kernel (see _GroupNormActFanout)."""
    w = gn.weight if gn.affine else None
    b = gn.bias if gn.affine else None
    return _GroupNormActFanout.apply(x, w, b, gn.num_groups, gn.eps, act)


def group_norm_act(x, gn: torch.nn.GroupNorm, act: int = ACT_SILU, bias_nc=None):
    """act(GroupNorm(x + bias_nc)) using the parameters of an nn.GroupNorm module."""
    w = gn.weight if gn.affine else None
    b = gn.bias if gn.affine else None
    return _GroupNormAct.apply(x, bias_nc, w, b, gn.num_groups, gn.eps, act)


def group_norm_act_f(x, num_groups, weight, bias, eps, act=ACT_SILU, bias_nc=None):
    return _GroupNormAct.apply(x, bias_nc, weight, bias, num_groups, eps, act)


def group_norm_affine_partials(part, N, C, gn: torch.nn.GroupNorm, bias_nc=None, part2=None):
    """(s, t) [N, C, 2] from partial statistics (part [N, C, R, 2], R, cnt) without touching
    the tensor; part2 given: the tensor is the channel concatenation of two whose partials
    are part (first C1 channels) and part2 (the rest), read in place."""
    pt, R, cnt = part
    ss = torch.empty((N, C, 2), device=pt.device, dtype=torch.float32)
    bnc = bias_nc.contiguous() if bias_nc is not None else None
    w = gn.weight if gn.affine else None
    b = gn.bias if gn.affine else None
    wp = w.detach().data_ptr() if w is not None else None
    bp = b.detach().data_ptr() if b is not None else None
    bncp = bnc.data_ptr() if bnc is not None else None
    if part2 is None:
        check(lib.bpk_group_norm_affine_partials_f32(
            pt.data_ptr(), R, cnt, bncp, wp, bp, ss.data_ptr(), N, C, gn.num_groups,
            float(gn.eps), stream_ptr(pt.device)), "group_norm_affine_partials")
        return ss
    pt2, R2, cnt2 = part2
    C1 = pt.shape[1]
    if (R2, cnt2) != (R, cnt) or pt.shape[0] != N or pt2.shape[:2] != (N, C - C1):
        raise RuntimeError("group_norm_affine_partials: mismatched partials of the two parts")
    check(lib.bpk_group_norm_affine_partials2_f32(
        pt.data_ptr(), C1, pt2.data_ptr(), R, cnt, bncp, wp, bp, ss.data_ptr(), N, C,
        gn.num_groups, float(gn.eps), stream_ptr(pt.device)), "group_norm_affine_partials2")
    return ss


def group_norm_affine(x, gn: torch.nn.GroupNorm, bias_nc=None):
    """Per-(n, c) (scale, shift) [N, C, 2] with act(GN(x + bias_nc)) == act(x * s + t):
    the statistics pass of GroupNorm alone (one read of x), for convolutions that apply the
    normalization in their input load (op.conv.conv3x3(..., pre=)).  Inference only."""
    require_hip(x, bias_nc, what="group_norm_affine")
    from .conv import gn_partials
    part = gn_partials(x)
    if part is not None:  # statistics from the producing conv's epilogue: no pass over x
        return group_norm_affine_partials(part, x.shape[0], x.shape[1], gn, bias_nc)
    x = x.contiguous()
    N, C = x.shape[:2]
    HW = x.numel() // max(N * C, 1)
    G = gn.num_groups
    ss = torch.empty((N, C, 2), device=x.device, dtype=torch.float32)
    ws = _ws(N, C, HW, G, x.device)
    bnc = bias_nc.contiguous() if bias_nc is not None else None
    w = gn.weight if gn.affine else None
    b = gn.bias if gn.affine else None
    check(lib.bpk_group_norm_affine_f32(
        x.data_ptr(), bnc.data_ptr() if bnc is not None else None,
        w.detach().data_ptr() if w is not None else None,
        b.detach().data_ptr() if b is not None else None, ss.data_ptr(),
        ws.data_ptr() if ws is not None else None, N, C, HW, G, float(gn.eps),
        stream_ptr(x.device)), "group_norm_affine")
    return ss


def group_norm_affine_stats(x, num_groups, weight, bias, eps, bias_nc=None):
    """(ss [N, C, 2], mean [N, G], rstd [N, G]): the affine form of SiLU(GroupNorm(x + bias_nc))
    (as group_norm_affine) plus the group statistics it was built from, for the backward of a
    conv that applied it in its input load (op.conv.gn_silu_conv3x3_ad).  From the producer's
    partial statistics when x carries them (no pass over x), else one read of x."""
    require_hip(x, bias_nc, what="group_norm_affine_stats")
    from .conv import gn_partials
    x = x.contiguous() if gn_partials(x) is None else x
    N, C = x.shape[:2]
    G = num_groups
    HW = x.numel() // max(N * C, 1)
    ss = torch.empty((N, C, 2), device=x.device, dtype=torch.float32)
    mean = torch.empty((N, G), device=x.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    bnc = bias_nc.detach().contiguous() if bias_nc is not None else None
    wp = weight.detach().data_ptr() if weight is not None else None
    bp = bias.detach().data_ptr() if bias is not None else None
    bncp = bnc.data_ptr() if bnc is not None else None
    part = gn_partials(x)
    if part is not None:
        pt, R, cnt = part
        check(lib.bpk_group_norm_affine_partials_stats_f32(
            pt.data_ptr(), R, cnt, bncp, wp, bp, ss.data_ptr(), mean.data_ptr(),
            rstd.data_ptr(), N, C, G, float(eps), stream_ptr(x.device)),
            "group_norm_affine_partials_stats")
    else:
        ws = _ws(N, C, HW, G, x.device)
        check(lib.bpk_group_norm_affine_stats_f32(
            x.data_ptr(), bncp, wp, bp, ss.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
            ws.data_ptr() if ws is not None else None, N, C, HW, G, float(eps),
            stream_ptr(x.device)), "group_norm_affine_stats")
    return ss, mean, rstd


def affine_silu(x, ss):
    """silu(x * s + t) for ss [N, C, 2] = (s, t): the activation the Winograd conv's GroupNorm
    prologue computes, materialised (for the conv's weight gradient)."""
    require_hip(x, ss, what="affine_silu")
    x = x.contiguous()
    N, C = x.shape[:2]
    y = torch.empty_like(x)
    check(lib.bpk_affine_silu_f32(x.data_ptr(), ss.contiguous().data_ptr(), y.data_ptr(), N, C,
                                  x.numel() // max(N * C, 1), stream_ptr(x.device)),
          "affine_silu")
    return y


class _Residual(Function):
    @staticmethod
    def forward(ctx, x, h, bias, div):
        mark_inputs(ctx, x, h, bias, div)
        require_hip(x, h, what="residual_rescale")
        x, h = x.contiguous(), h.contiguous()
        if x.shape != h.shape:
            raise RuntimeError(f"residual_rescale: shape mismatch {x.shape} vs {h.shape}")
        N, C = x.shape[:2]
        HW = x.numel() // max(N * C, 1)
        out = torch.empty_like(x)
        check(lib.bpk_residual_rescale_f32(x.data_ptr(), h.data_ptr(),
                                           bias.data_ptr() if bias is not None else None,
                                           out.data_ptr(), N, C, HW, float(div),
                                           stream_ptr(x.device)), "residual_rescale")
        ctx.div = div
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, g):
        gd = g / ctx.div
        gb = gd.sum(dim=[0] + list(range(2, g.ndim))) if ctx.has_bias and want_grad(ctx, 2) \
            else None
        return gd, gd, gb, None


def residual_rescale(x, h, bias=None, div=2 ** 0.5):
    return _Residual.apply(x, h, bias, div)


# ------------------------------------------------ InstanceNorm2d + ELU, twice differentiable

ACT_ELU = 1


def _in_fns(dtype):
    if dtype == torch.float32:
        return (lib.bpk_instance_norm_act_fwd_f32, lib.bpk_instance_norm_act_bwd_f32,
                lib.bpk_instance_norm_act_bwd2_f32)
    if dtype == torch.float64:
        return (lib.bpk_instance_norm_act_fwd_f64, lib.bpk_instance_norm_act_bwd_f64,
                lib.bpk_instance_norm_act_bwd2_f64)
    raise RuntimeError(f"instance_norm_act: float32 / float64 only, got {dtype}")


def _planes(x):
    if x.dim() < 3:
        raise RuntimeError(f"instance_norm_act: expected [N, C, ...], got {tuple(x.shape)}")
    return x.shape[0] * x.shape[1], x[0, 0].numel()


class _InstanceNormAct(Function):
    """y = act(InstanceNorm(x)) (affine=False, instance statistics).  Its backward is
    _InstanceNormActBackward, whose own backward is the analytic double backward -- the
    PINN residual's second derivatives through PressureNet (csrc/instance_norm.hip)."""

    @staticmethod
    def forward(ctx, x, eps, act):
        require_hip(x, what="instance_norm_act")
        P, M = _planes(x)
        y = torch.empty_like(x)
        mean = torch.empty(P, device=x.device, dtype=x.dtype)
        rstd = torch.empty_like(mean)
        check(_in_fns(x.dtype)[0](x.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                  P, M, float(eps), act, stream_ptr(x.device)),
              "instance_norm_act_fwd")
        ctx.save_for_backward(x, mean, rstd)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd = ctx.saved_tensors
        return _InstanceNormActBackward.apply(dy.contiguous(), x, mean, rstd, ctx.act), None, None


class _InstanceNormActBackward(Function):
    """dx = d act(IN(x)) / dx applied to dy (+ add, the fan-out form's skip gradient, added in
    the same kernel pass); differentiable once more (w.r.t. dy and x; mean and rstd are
    functions of x already accounted for by the double-backward kernel; w.r.t. add: identity)."""

    @staticmethod
    def forward(ctx, dy, x, mean, rstd, act, add=None):
        P, M = _planes(x)
        dx = torch.empty_like(x)
        if add is not None and x.dtype == torch.float32:
            add = add.contiguous()
            check(lib.bpk_instance_norm_act_bwd_add_f32(
                dy.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), add.data_ptr(),
                dx.data_ptr(), P, M, act, stream_ptr(x.device)), "instance_norm_act_bwd_add")
        else:
            check(_in_fns(x.dtype)[1](dy.data_ptr(), x.data_ptr(), mean.data_ptr(),
                                      rstd.data_ptr(), dx.data_ptr(), P, M, act,
                                      stream_ptr(x.device)), "instance_norm_act_bwd")
            if add is not None:  # float64 (gradcheck): the plain sum
                dx.add_(add)
        ctx.save_for_backward(dy, x, mean, rstd)
        ctx.act = act
        return dx

    @staticmethod
    @once_differentiable
    def backward(ctx, v, *_):
        dy, x, mean, rstd = ctx.saved_tensors
        need_dy, need_x = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        need_add = len(ctx.needs_input_grad) > 5 and ctx.needs_input_grad[5]
        P, M = _planes(x)
        v = v.contiguous()
        gdy = torch.empty_like(x) if need_dy else None
        gx = torch.empty_like(x) if need_x else None
        check(_in_fns(x.dtype)[2](v.data_ptr(), dy.data_ptr(), x.data_ptr(), mean.data_ptr(),
                                  rstd.data_ptr(), gdy.data_ptr() if gdy is not None else None,
                                  gx.data_ptr() if gx is not None else None, P, M, ctx.act,
                                  stream_ptr(x.device)), "instance_norm_act_bwd2")
        return gdy, gx, None, None, None, (v if need_add else None)


class _InstanceNormActFanout(Function):
    """(act(IN(x)), x): for a residual block whose input feeds both its first norm and its
    skip.  Both gradients reach this one node, and the skip's is added inside the norm's
    backward kernel (bpk_instance_norm_act_bwd_add_f32) -- no accumulation launch of autograd's
    -- in every derivative pass of the PINN residual (the first-order pass records the fused
    backward, whose own backward hands the addend's gradient through unchanged)."""

    @staticmethod
    def forward(ctx, x, eps, act):
        require_hip(x, what="instance_norm_act")
        ctx.set_materialize_grads(False)
        P, M = _planes(x)
        y = torch.empty_like(x)
        mean = torch.empty(P, device=x.device, dtype=x.dtype)
        rstd = torch.empty_like(mean)
        check(_in_fns(x.dtype)[0](x.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                  P, M, float(eps), act, stream_ptr(x.device)),
              "instance_norm_act_fwd")
        ctx.save_for_backward(x, mean, rstd)
        ctx.act = act
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dskip):
        x, mean, rstd = ctx.saved_tensors
        if dy is None:
            return dskip, None, None
        return (_InstanceNormActBackward.apply(dy.contiguous(), x, mean, rstd, ctx.act, dskip),
                None, None)


def instance_norm_act_fanout(x, eps=1e-5, act=ACT_ELU):
    """(act(F.instance_norm(x, eps=eps)), x) -- the skip's gradient joins the norm's inside the
    backward kernel (see _InstanceNormActFanout)."""
    require_hip(x, what="instance_norm_act")
    return _InstanceNormActFanout.apply(x.contiguous(), float(eps), int(act))


def instance_norm_act(x, eps=1e-5, act=ACT_ELU):
    """act(F.instance_norm(x, eps=eps)) for x [N, C, H, W] on HIP (act: ACT_ELU or 0).
    The input is made dense as a recorded op, outside the Function (a copy made inside
    and saved would cut the double backward from the graph)."""
    require_hip(x, what="instance_norm_act")
    return _InstanceNormAct.apply(x.contiguous(), float(eps), int(act))
