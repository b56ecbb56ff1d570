"""FIR up/down-sampling layers (StyleGAN2 style) on the HIP upfirdn2d kernel.

Reference: models/up_or_down_sampling.py.  Same public functions and `Conv2d`
module (parameters `weight` [out, in, k, k], `bias` [out]).  Differences:
  * the FIR taps are built once per (kernel, gain, device) and cached on the
    device instead of `torch.tensor(k, device=...)` on every call (an H2D copy
    per call in the reference, e.g. up_or_down_sampling.py:223);
  * `upsample_conv_2d` flips the weight with `torch.flip` -- the reference's
    negative-step slice (up_or_down_sampling.py:126) raises in PyTorch, so that
    path is unreachable there; parity unpinned.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from op import conv as conv_op
from op import upfirdn2d

_KERNEL_CACHE: dict = {}


def _setup_kernel(k):
    k = np.asarray(k, dtype=np.float32)
    if k.ndim == 1:
        k = np.outer(k, k)
    k /= np.sum(k)
    assert k.ndim == 2 and k.shape[0] == k.shape[1]
    return k


def fir_kernel(k, scale, device, dtype=torch.float32):
    """Cached device tensor of `_setup_kernel(k) * scale`."""
    key = (tuple(np.asarray(k, dtype=np.float64).ravel().tolist()), np.asarray(k).ndim, float(scale),
           str(device), dtype)
    t = _KERNEL_CACHE.get(key)
    if t is None:
        arr = _setup_kernel(k) * scale
        t = torch.tensor(arr, device=device, dtype=dtype)
        _KERNEL_CACHE[key] = t
    return t


class Conv2d(nn.Module):
    """Conv2d with optional fused FIR up/down-sampling (reference :23-56)."""

    def __init__(self, in_ch, out_ch, kernel, up=False, down=False, resample_kernel=(1, 3, 3, 1),
                 use_bias=True, kernel_init=None):
        super().__init__()
        assert not (up and down)
        assert kernel >= 1 and kernel % 2 == 1
        self.weight = nn.Parameter(torch.zeros(out_ch, in_ch, kernel, kernel))
        if kernel_init is not None:
            self.weight.data = kernel_init(self.weight.data.shape)
        if use_bias:
            self.bias = nn.Parameter(torch.zeros(out_ch))
        self.up, self.down = up, down
        self.resample_kernel = resample_kernel
        self.kernel = kernel
        self.use_bias = use_bias

    def forward(self, x):
        b = self.bias if self.use_bias else None
        if self.up:
            x = upsample_conv_2d(x, self.weight, k=self.resample_kernel)
            return x + b.reshape(1, -1, 1, 1) if b is not None else x
        if self.down:
            return conv_downsample_2d(x, self.weight, k=self.resample_kernel, bias=b)
        return _conv(x, self.weight, b, 1, self.kernel // 2)


def _native(x):
    return x.is_cuda and x.dtype == torch.float32


def _conv(x, w, bias, stride, padding):
    """F.conv2d on the native kernels (op.conv: Winograd / implicit-GEMM MFMA, every
    derivative order a plain convolution) for fp32 HIP tensors."""
    if _native(x):
        if stride == 1 and padding == 1 and tuple(w.shape[2:]) == (3, 3):
            return conv_op.conv3x3(x, w, bias)
        return conv_op.conv2d_general(x, w, bias, stride, padding)
    return F.conv2d(x, w, bias, stride=stride, padding=padding)


def naive_upsample_2d(x, factor=2):
    _N, C, H, W = x.shape
    x = torch.reshape(x, (-1, C, H, 1, W, 1)).repeat(1, 1, 1, factor, 1, factor)
    return torch.reshape(x, (-1, C, H * factor, W * factor))


def naive_downsample_2d(x, factor=2):
    _N, C, H, W = x.shape
    x = torch.reshape(x, (-1, C, H // factor, factor, W // factor, factor))
    return torch.mean(x, dim=(3, 5))


def upsample_conv_2d(x, w, k=None, factor=2, gain=1):
    """Transposed strided conv followed by the FIR (reference :72-141)."""
    assert isinstance(factor, int) and factor >= 1
    assert w.ndim == 4
    convH, convW = w.shape[2], w.shape[3]
    inC, outC = w.shape[1], w.shape[0]
    assert convW == convH
    kk = [1] * factor if k is None else k
    ksz = _setup_kernel(kk).shape[0]
    p = (ksz - factor) - (convW - 1)
    num_groups = x.shape[1] // inC
    out_h = (x.shape[2] - 1) * factor + convH
    out_w = (x.shape[3] - 1) * factor + convW
    op = (out_h - (x.shape[2] - 1) * factor - convH, out_w - (x.shape[3] - 1) * factor - convW)
    wt = torch.reshape(w, (num_groups, -1, inC, convH, convW))
    wt = torch.flip(wt, [3, 4]).permute(0, 2, 1, 3, 4)
    wt = torch.reshape(wt, (num_groups * inC, -1, convH, convW))
    if _native(x):
        x = conv_op.conv_transpose2d_general(x, wt, None, factor, 0, op)
    else:
        x = F.conv_transpose2d(x, wt, stride=(factor, factor), output_padding=op, padding=0)
    kt = fir_kernel(kk, gain * (factor ** 2), x.device, x.dtype)
    return upfirdn2d(x, kt, pad=((p + 1) // 2 + factor - 1, p // 2 + 1))


def conv_downsample_2d(x, w, k=None, factor=2, gain=1, bias=None):
    """FIR then strided conv (reference :144-178)."""
    assert isinstance(factor, int) and factor >= 1
    _outC, _inC, convH, convW = w.shape
    assert convW == convH
    kk = [1] * factor if k is None else k
    kt = fir_kernel(kk, gain, x.device, x.dtype)
    p = (kt.shape[0] - factor) + (convW - 1)
    x = upfirdn2d(x, kt, pad=((p + 1) // 2, p // 2))
    return _conv(x, w, bias, factor, 0)


def upsample_2d(x, k=None, factor=2, gain=1):
    """FIR upsampling (reference :195-224)."""
    assert isinstance(factor, int) and factor >= 1
    kk = [1] * factor if k is None else k
    kt = fir_kernel(kk, gain * (factor ** 2), x.device, x.dtype)
    p = kt.shape[0] - factor
    return upfirdn2d(x, kt, up=factor, pad=((p + 1) // 2 + factor - 1, p // 2))


def downsample_2d(x, k=None, factor=2, gain=1):
    """FIR downsampling (reference :227-257)."""
    assert isinstance(factor, int) and factor >= 1
    kk = [1] * factor if k is None else k
    kt = fir_kernel(kk, gain, x.device, x.dtype)
    p = kt.shape[0] - factor
    return upfirdn2d(x, kt, down=factor, pad=((p + 1) // 2, p // 2))
