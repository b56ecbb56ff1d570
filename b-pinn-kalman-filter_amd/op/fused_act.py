"""`op.fused_leaky_relu` / `op.FusedLeakyReLU` on the HIP kernel (csrc/fused_bias_act.hip).

Reference: op/fused_act.py:20-97 + op/fused_bias_act_kernel.cu:18-98.
y = scale * leaky_relu(x + bias[c], negative_slope); the backward uses the output
sign as the mask (grad=1 mode, refer = out), grad_bias sums over every dim but 1,
and the double backward re-applies the same mask with the incoming bias grad
(op/fused_act.py:43-49).

Note: the reference's CPU branch hard-codes slope 0.2 (op/fused_act.py:91); this
build has no CPU branch and always honours `negative_slope`, matching the
reference's GPU semantics.

`leaky_relu` / `LeakyReLU`: the plain activation (no bias, scale 1) of FlowNet (reference
models/flownet.py: nn.LeakyReLU(0.1) after every conv, F.leaky_relu of the cost volume) on the
same kernel, bit-identical to aten's (out > 0 selects the same branch as x > 0 for a positive
slope).  Its backward is a Function of the output gradient only: the mask is piecewise constant,
so its derivative w.r.t. the activation is zero -- which aten's leaky_relu_backward
materializes (zeros_like + an accumulating add per node) on every pass of the PINN residual's
double backward.
"""
from __future__ import annotations

import torch
from torch import nn
from torch.autograd import Function

from ._lib import check, lib, require_hip, stream_ptr


def fused_bias_act_raw(x, bias, refer, act, grad, alpha, scale):
    """Mirror of the extension call `fused.fused_bias_act(x, bias, refer, act, grad, alpha, scale)`
    (op/fused_bias_act.cpp:11-20).  Empty bias/refer tensors mean "absent"."""
    require_hip(x, what="fused_bias_act")
    x = x.contiguous()
    use_b = bias is not None and bias.numel() > 0
    use_r = refer is not None and refer.numel() > 0
    b = bias.contiguous() if use_b else None
    r = refer.contiguous() if use_r else None
    step_b = 1
    for d in x.shape[2:]:
        step_b *= d
    out = torch.empty_like(x)
    if x.dtype == torch.float32:
        fn = lib.bpk_fused_bias_act_f32
    elif x.dtype == torch.float64:
        fn = lib.bpk_fused_bias_act_f64
    else:
        raise RuntimeError(f"fused_bias_act: unsupported dtype {x.dtype}")
    check(fn(x.data_ptr(), b.data_ptr() if use_b else None, r.data_ptr() if use_r else None,
             out.data_ptr(), x.numel(), step_b, b.numel() if use_b else 0, act, grad, float(alpha),
             float(scale), stream_ptr(x.device)), "fused_bias_act")
    return out


class _FusedLeakyReLUGrad(Function):
    @staticmethod
    def forward(ctx, grad_output, out, negative_slope, scale):
        ctx.save_for_backward(out)
        ctx.negative_slope, ctx.scale = negative_slope, scale
        grad_input = fused_bias_act_raw(grad_output, None, out, 3, 1, negative_slope, scale)
        dims = [0] + list(range(2, grad_input.ndim))
        grad_bias = grad_input.sum(dims).detach()
        return grad_input, grad_bias

    @staticmethod
    def backward(ctx, gg_input, gg_bias):
        out, = ctx.saved_tensors
        gg_out = fused_bias_act_raw(gg_input, gg_bias, out, 3, 1, ctx.negative_slope, ctx.scale)
        return gg_out, None, None, None


class _FusedLeakyReLUFn(Function):
    @staticmethod
    def forward(ctx, x, bias, negative_slope, scale):
        out = fused_bias_act_raw(x, bias, None, 3, 0, negative_slope, scale)
        ctx.save_for_backward(out)
        ctx.negative_slope, ctx.scale = negative_slope, scale
        return out

    @staticmethod
    def backward(ctx, grad_output):
        out, = ctx.saved_tensors
        gi, gb = _FusedLeakyReLUGrad.apply(grad_output.contiguous(), out, ctx.negative_slope,
                                           ctx.scale)
        return gi, gb, None, None


class _LeakyReLUGrad(Function):
    """g * (out > 0 ? 1 : slope): the backward of leaky_relu, linear in g (its own backward is
    itself), no gradient w.r.t. the mask source `out`."""

    @staticmethod
    def forward(ctx, g, out, negative_slope):
        ctx.save_for_backward(out)
        ctx.negative_slope = negative_slope
        return fused_bias_act_raw(g, None, out, 3, 1, negative_slope, 1.0)

    @staticmethod
    def backward(ctx, gg):
        out, = ctx.saved_tensors
        return _LeakyReLUGrad.apply(gg.contiguous(), out, ctx.negative_slope), None, None


class _LeakyReLU(Function):
    @staticmethod
    def forward(ctx, x, negative_slope):
        out = fused_bias_act_raw(x, None, None, 3, 0, negative_slope, 1.0)
        ctx.save_for_backward(out)
        ctx.negative_slope = negative_slope
        return out

    @staticmethod
    def backward(ctx, g):
        out, = ctx.saved_tensors
        return _LeakyReLUGrad.apply(g.contiguous(), out, ctx.negative_slope), None


def leaky_relu(input, negative_slope=0.01):
    """F.leaky_relu(input, negative_slope) on the native kernel, differentiable to any order."""
    require_hip(input, what="leaky_relu")
    if negative_slope <= 0:
        raise RuntimeError("leaky_relu: the output-sign mask needs negative_slope > 0")
    return _LeakyReLU.apply(input, float(negative_slope))


class LeakyReLU(nn.Module):
    """nn.LeakyReLU(negative_slope) on the native kernel (no parameters, no state-dict keys)."""

    def __init__(self, negative_slope=0.01, inplace=False):
        super().__init__()
        self.negative_slope = negative_slope

    def forward(self, input):
        return leaky_relu(input, self.negative_slope)

    def extra_repr(self):
        return f"negative_slope={self.negative_slope}"


def fused_leaky_relu(input, bias, negative_slope=0.2, scale=2 ** 0.5):
    require_hip(input, bias, what="fused_leaky_relu")
    return _FusedLeakyReLUFn.apply(input, bias, negative_slope, scale)


class FusedLeakyReLU(nn.Module):
    def __init__(self, channel, negative_slope=0.2, scale=2 ** 0.5):
        super().__init__()
        self.bias = nn.Parameter(torch.zeros(channel))
        self.negative_slope = negative_slope
        self.scale = scale

    def forward(self, input):
        return fused_leaky_relu(input, self.bias, self.negative_slope, self.scale)
