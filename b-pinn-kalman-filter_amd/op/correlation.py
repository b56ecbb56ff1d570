"""FlowNet cost volume on the gfx950 kernels of csrc/correlation.hip.

Same API as the reference's CuPy op (op/correlation.py:291-487):
`FunctionCorrelation(tensorFirst, tensorSecond, stride)` and `ModuleCorrelation`,
returning [B, 49, ceil(H/stride), ceil(W/stride)].  As in the reference, the
backward produces plain tensors (no graph), so second-order terms through the
correlation are constant -- kept for parity with
`PINN.equation_mse`.  Inputs must be contiguous (the reference asserts it, :310-311)
and on a HIP device (the reference raises NotImplementedError on CPU, :377).
"""
from __future__ import annotations

import torch

from ._lib import check, lib, require_hip, stream_ptr


def correlation_fwd_raw(first, second, stride: int):
    B, C, H, W = first.shape
    out = first.new_empty((B, 49, -(-H // stride), -(-W // stride)))
    check(lib.bpk_correlation_fwd_f32(first.data_ptr(), second.data_ptr(), out.data_ptr(), B, C,
                                      H, W, stride, stream_ptr(first.device)), "correlation")
    return out


def correlation_bwd_raw(first, second, grad_out, stride: int, need_first=True,
                        need_second=True):
    B, C, H, W = first.shape
    gf = torch.empty_like(first) if need_first else None
    gs = torch.empty_like(first) if need_second else None
    check(lib.bpk_correlation_bwd_f32(first.data_ptr(), second.data_ptr(), grad_out.data_ptr(),
                                      None if gf is None else gf.data_ptr(),
                                      None if gs is None else gs.data_ptr(), B, C, H, W, stride,
                                      stream_ptr(first.device)), "correlation_bwd")
    return gf, gs


class _FunctionCorrelation(torch.autograd.Function):
    @staticmethod
    def forward(ctx, first, second, intStride):
        assert first.is_contiguous() and second.is_contiguous()
        assert first.shape == second.shape and first.dim() == 4
        if first.dtype != torch.float32:
            raise RuntimeError(f"correlation: float32 only (got {first.dtype})")
        ctx.save_for_backward(first, second)
        ctx.intStride = intStride
        return correlation_fwd_raw(first, second, intStride)

    @staticmethod
    def backward(ctx, gradOutput):
        first, second = ctx.saved_tensors
        with torch.no_grad():
            gf, gs = correlation_bwd_raw(first, second, gradOutput.detach().contiguous(), ctx.intStride,
                                         ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        return gf, gs, None


def FunctionCorrelation(tensorFirst, tensorSecond, stride):
    require_hip(tensorFirst, tensorSecond, what="correlation")
    return _FunctionCorrelation.apply(tensorFirst, tensorSecond, stride)


class ModuleCorrelation(torch.nn.Module):
    def forward(self, tensorFirst, tensorSecond, stride):
        return FunctionCorrelation(tensorFirst, tensorSecond, stride)
