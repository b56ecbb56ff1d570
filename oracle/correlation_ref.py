"""ORACLE (test infrastructure only) -- FlowNet correlation restated in numpy.

Follows the reference's CuPy kernels (op/correlation.py): inputs are zero-padded
by 3*stride exactly as `kernel_Correlation_rearrange` does (:13-31, padded
tensors allocated :296-306); the forward is `kernel_Correlation_updateOutput`
(:34-102: mean over channels of first * shifted second, displacement index
(dy+3)*7 + (dx+3), output ceil(H/s) x ceil(W/s), :317-321); the grads follow
`kernel_Correlation_updateGrad{First,Second}` (:104-231) including their
ceil/floor range arithmetic.  Sums are accumulated in float64 and rounded once,
so GPU results are compared with a float32 tolerance (float64 inputs give float64 outputs:
the float64-truth fixtures, tests/golden/make_golden_pinn_f64.py).  No runnable reference
exists here (CuPy/CUDA only): pinned by known-answer tests in tests/test_oracle.py.
"""
from __future__ import annotations

import numpy as np


def _pad(a, s):
    p = 3 * s
    return np.pad(a.astype(np.float64), ((0, 0), (0, 0), (p, p), (p, p)))


def _out_dtype(a):
    return np.float64 if a.dtype == np.float64 else np.float32


def forward(first, second, stride=1):
    B, C, H, W = first.shape
    s = stride
    Ho, Wo = -(-H // s), -(-W // s)
    f1, f2 = _pad(first, s), _pad(second, s)
    out = np.zeros((B, 49, Ho, Wo))
    ys = (np.arange(Ho) + 3) * s          # x1/y1 of the reference (:49-50), padded coords
    xs = (np.arange(Wo) + 3) * s
    a = f1[:, :, ys][:, :, :, xs]
    for tc in range(49):
        s2o = (tc % 7 - 3) * s
        s2p = (tc // 7 - 3) * s
        b = f2[:, :, ys + s2p][:, :, :, xs + s2o]
        out[:, tc] = (a * b).sum(1) / C
    return out.astype(_out_dtype(first))


def backward(first, second, gout, stride=1):
    """(grad_first, grad_second) of `forward` for upstream gradient gout."""
    B, C, H, W = first.shape
    s = stride
    Ho, Wo = gout.shape[2], gout.shape[3]
    f1, f2 = _pad(first, s), _pad(second, s)
    g = gout.astype(np.float64)
    gf = np.zeros((B, C, H, W))
    gs = np.zeros((B, C, H, W))
    for m0 in range(H):           # h-pos (unpadded); m = m0 + 3s in the reference
        for l0 in range(W):
            # grad first (:116-160): x range ceil(l0/s)..floor(l0/s)
            if l0 % s == 0 and m0 % s == 0 and l0 // s < Wo and m0 // s < Ho:
                oy, ox = m0 // s, l0 // s
                acc = np.zeros((B, C))
                for p in range(-3, 4):
                    for o in range(-3, 4):
                        op = (p + 3) * 7 + (o + 3)
                        acc += g[:, op, oy, ox][:, None] * f2[:, :, m0 + 3 * s + p * s,
                                                            l0 + 3 * s + o * s]
                gf[:, :, m0, l0] = acc / C
            # grad second (:179-225)
            acc = np.zeros((B, C))
            for p in range(-3, 4):
                for o in range(-3, 4):
                    xo, yo = l0 - o * s, m0 - p * s
                    if xo % s or yo % s:
                        continue
                    ox, oy = xo // s, yo // s
                    if ox < 0 or oy < 0 or ox >= Wo or oy >= Ho:
                        continue
                    op = (p + 3) * 7 + (o + 3)
                    acc += g[:, op, oy, ox][:, None] * f1[:, :, yo + 3 * s, xo + 3 * s]
            gs[:, :, m0, l0] = acc / C
    return gf.astype(_out_dtype(first)), gs.astype(_out_dtype(first))
