"""Small GEMMs of the score networks on the native strided batched MFMA GEMM
(csrc/gemm_strided.hip, `bpk_gemm_sb_f32`): `linear` for nn.Linear (the time-embedding MLP
and the residual blocks' Dense_0, reference models/ncsnpp.py:86-89, layerspp.py:232-262) and
`bmm` for the attention block's two batched products under autograd (reference
layerspp.py:84-88).  Both are autograd Functions whose gradients are the same kernel with
transposed strides (no copies), so every derivative order stays native."""
from __future__ import annotations

import torch

from . import flops
from ._lib import check, lib, require_hip, stream_ptr


def _strides3(t):
    """(batch, row, col) element strides of a 3-D view (a 2-D one as batch 1)."""
    if t.dim() == 2:
        return (0,) + tuple(t.stride())
    return tuple(t.stride())


def gemm_sb(a, b, bias=None, bias_mode=0, alpha=1.0, out=None):
    """C[i] = alpha a[i] @ b[i] (+ bias) for 3-D (or 2-D) float32 HIP views of any strides;
    returns a new contiguous C (or accumulates into `out`)."""
    require_hip(a, b, bias, what="gemm_sb")
    if a.dtype != torch.float32 or b.dtype != torch.float32:
        raise RuntimeError("gemm_sb: float32 operands only")
    two = a.dim() == 2 and b.dim() == 2
    a3 = a if a.dim() == 3 else a.unsqueeze(0)
    b3 = b if b.dim() == 3 else b.unsqueeze(0)
    ba, bb = a3.shape[0], b3.shape[0]
    if a3.dim() != 3 or b3.dim() != 3 or not (ba == bb or ba == 1 or bb == 1):
        raise RuntimeError(f"gemm_sb: batch sizes {tuple(a.shape)} x {tuple(b.shape)} "
                           "(equal, or one of them 1 and broadcast)")
    batch = max(ba, bb)
    M, K = a3.shape[1], a3.shape[2]
    if b3.shape[1] != K:
        raise RuntimeError(f"gemm_sb: inner sizes {tuple(a.shape)} x {tuple(b.shape)}")
    N = b3.shape[2]
    sa = (0 if ba == 1 else a3.stride(0),) + tuple(a3.stride()[1:])
    sb = (0 if bb == 1 else b3.stride(0),) + tuple(b3.stride()[1:])
    acc = out is not None
    if acc:
        want = (M, N) if (two and out.dim() == 2) else (batch, M, N)
        if (tuple(out.shape) != want or out.dtype != torch.float32 or not out.is_cuda
                or out.device != a.device):
            raise RuntimeError(f"gemm_sb: out {tuple(out.shape)} {out.dtype} on {out.device}, "
                               f"expected float32 {want} on {a.device}")
    c = out if acc else torch.empty((batch, M, N), dtype=torch.float32, device=a.device)
    c3 = c if c.dim() == 3 else c.unsqueeze(0)
    bias_c = None if bias is None else bias.detach().contiguous()
    if (bias_c is not None and bias_mode in (1, 2)
            and bias_c.numel() != (N if bias_mode == 1 else M)):
        raise RuntimeError(f"gemm_sb: bias of {bias_c.numel()} values for bias_mode {bias_mode} "
                           f"(M {M}, N {N})")
    check(lib.bpk_gemm_sb_f32(a3.data_ptr(), *sa, b3.data_ptr(), *sb, c3.data_ptr(),
                              *_strides3(c3), None if bias_c is None else bias_c.data_ptr(),
                              bias_mode if bias_c is not None else 0, float(alpha), int(acc),
                              batch, M, N, K, stream_ptr(a.device)), "gemm_sb")
    flops.add("gemm_sb", 2.0 * batch * M * N * K)
    if acc:
        return out
    return c[0] if two else c


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        x2 = x.reshape(-1, x.shape[-1])
        y = gemm_sb(x2, weight.t(), bias, 1)  # [rows, out] = x W^T + b
        return y.reshape(x.shape[:-1] + (weight.shape[0],))

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = linear(gy, weight.t())                      # gy W
        if ctx.needs_input_grad[1]:
            g2 = gy.reshape(-1, gy.shape[-1])
            gw = bmm_ad(g2.t(), x.reshape(-1, x.shape[-1]))  # gy^T x
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = gy.reshape(-1, gy.shape[-1]).sum(0)
        return gx, gw, gb


def linear(x, weight, bias=None):
    """F.linear(x, weight, bias) on the native GEMM, differentiable to any order."""
    require_hip(x, weight, bias, what="linear")
    return _Linear.apply(x, weight, bias)


class _Bmm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return gemm_sb(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ga = gb = None
        if ctx.needs_input_grad[0]:
            ga = bmm_ad(g, b.transpose(-1, -2))
        if ctx.needs_input_grad[1]:
            gb = bmm_ad(a.transpose(-1, -2), g)
        return ga, gb


def bmm_ad(a, b):
    """torch.bmm(a, b) (or mm for 2-D) on the native GEMM, differentiable to any order;
    transposed views are read through their strides."""
    require_hip(a, b, what="bmm")
    return _Bmm.apply(a, b)


def supported(*tensors) -> bool:
    return all(t is None or (t.is_cuda and t.dtype == torch.float32) for t in tensors)
