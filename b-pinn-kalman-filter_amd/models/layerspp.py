"""NCSN++ layers on the gfx950 path (reference: models/layerspp.py).

Module / parameter names are the reference's (GroupNorm_0, Conv_0, Dense_0,
GroupNorm_1, Conv_1, Conv_2, NIN_*, Conv2d_0, W) so reference state dicts load.
Per block the arithmetic is re-scheduled for the GPU:
  GroupNorm_0+SiLU                  -> 1 fused launch
  FIR up/down of h and x            -> upfirdn2d HIP kernel
  Conv_0 (no bias)                  -> conv
  + Conv_0.bias + Dense_0(SiLU(temb)), GroupNorm_1, SiLU -> 1 fused launch
  Conv_1 (no bias), + Conv_1.bias + skip, / sqrt(2)      -> conv + 1 fused launch
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from op.norm_act import residual_rescale

from . import layers, up_or_down_sampling

# attention at inference: q, k, v as one GEMM over the stacked NIN weights
_ATTN_QKV = True
# ... and softmax(q^T k) v as one fused kernel (csrc/attention.hip; False: bmm + softmax + bmm)
_ATTN_FUSED = True

conv1x1 = layers.ddpm_conv1x1
conv3x3 = layers.ddpm_conv3x3
NIN = layers.NIN
default_init = layers.default_init
gn_act = layers.gn_act
conv_nobias = layers.conv_nobias


class GaussianFourierProjection(nn.Module):
    """Random Fourier features of log-sigma (reference :32-41)."""

    def __init__(self, embedding_size=256, scale=1.0):
        super().__init__()
        self.W = nn.Parameter(torch.randn(embedding_size) * scale, requires_grad=False)

    def forward(self, x):
        proj = x[:, None] * self.W[None, :] * 2 * np.pi
        return torch.cat([torch.sin(proj), torch.cos(proj)], dim=-1)


class Combine(nn.Module):
    """1x1 conv of x then concat/sum with y (reference :44-59)."""

    def __init__(self, dim1, dim2, method="cat"):
        super().__init__()
        self.Conv_0 = conv1x1(dim1, dim2)
        self.method = method

    def forward(self, x, y):
        h = self.Conv_0(x)
        if self.method == "cat":
            return torch.cat([h, y], dim=1)
        if self.method == "sum":
            return h + y
        raise ValueError(f"Method {self.method} not recognized.")


class AttnBlockpp(nn.Module):
    """Channel self-attention over H*W positions (reference :62-91)."""

    def __init__(self, channels, skip_rescale=False, init_scale=0.):
        super().__init__()
        self.GroupNorm_0 = nn.GroupNorm(num_groups=min(channels // 4, 32), num_channels=channels,
                                        eps=1e-6)
        self.NIN_0 = NIN(channels, channels)
        self.NIN_1 = NIN(channels, channels)
        self.NIN_2 = NIN(channels, channels)
        self.NIN_3 = NIN(channels, channels, init_scale=init_scale)
        self.skip_rescale = skip_rescale

    def forward(self, x):
        h = gn_act(x, self.GroupNorm_0, None)
        div = np.sqrt(2.) if self.skip_rescale else 1.0
        if _ATTN_QKV and not torch.is_grad_enabled() and self._qkv_ok(h):
            return residual_rescale(x, self._forward_qkv(h), None, div)
        h = self.NIN_3(layers._attention(h, self.NIN_0, self.NIN_1, self.NIN_2))
        return residual_rescale(x, h, None, div)

    def _qkv_ok(self, h):
        from op import conv as conv_op
        N, C, H, W = h.shape
        return (h.is_cuda and h.dtype == torch.float32
                and bool(conv_op.lib.bpk_gemm_nchw_supported(N, 3 * C, H * W, C, 0))
                and bool(conv_op.lib.bpk_gemm_nchw_supported(N, C, H * W, C, 0)))

    def _forward_qkv(self, h):
        """Inference: q, k, v as ONE MFMA GEMM over the stacked NIN weights, NIN_3 as another
        (op.conv.conv1x1), the 1/sqrt(C) scale folded into q's weights when it is a power of
        two (exact: C = 4^k, e.g. 256) and applied to the logits otherwise."""
        from op import conv as conv_op
        B, C, H, W = h.shape
        s = float(int(C) ** (-0.5))
        fold = math.frexp(s)[0] == 0.5  # s is a power of two
        sq = s if fold else 1.0
        wqkv = torch.cat([self.NIN_0.W.t() * sq, self.NIN_1.W.t(), self.NIN_2.W.t()], 0)
        bqkv = torch.cat([self.NIN_0.b * sq, self.NIN_1.b, self.NIN_2.b], 0)
        qkv = conv_op.conv1x1(h, wqkv, bqkv).reshape(B, 3, C, H * W)
        from op import attention as attn_op
        if _ATTN_FUSED and attn_op.supported(qkv):
            out = attn_op.attention(qkv, 1.0 if fold else s).reshape(B, C, H, W)
            return conv_op.conv1x1(out, self.NIN_3.W.t(), self.NIN_3.b)
        q, k, v = qkv[:, 0], qkv[:, 1], qkv[:, 2]
        w = torch.bmm(q.transpose(1, 2), k)
        if not fold:
            w = w * s
        w = torch.softmax(w, dim=-1)
        out = torch.bmm(v, w.transpose(1, 2)).reshape(B, C, H, W)
        return conv_op.conv1x1(out, self.NIN_3.W.t(), self.NIN_3.b)


class Upsample(nn.Module):
    """x2 upsampling: nearest(+conv) or FIR(+fused conv) (reference :94-126)."""

    def __init__(self, in_ch=None, out_ch=None, with_conv=False, fir=False,
                 fir_kernel=(1, 3, 3, 1)):
        super().__init__()
        out_ch = out_ch if out_ch else in_ch
        if not fir:
            if with_conv:
                self.Conv_0 = conv3x3(in_ch, out_ch)
        elif with_conv:
            self.Conv2d_0 = up_or_down_sampling.Conv2d(in_ch, out_ch, kernel=3, up=True,
                                                       resample_kernel=fir_kernel, use_bias=True,
                                                       kernel_init=default_init())
        self.fir, self.with_conv = fir, with_conv
        self.fir_kernel = fir_kernel
        self.out_ch = out_ch

    def forward(self, x):
        B, C, H, W = x.shape
        if not self.fir:
            # the reference passes 'nearest' positionally as scale_factor (layerspp.py:117),
            # which raises; the intended nearest-neighbour upsample is used here
            h = F.interpolate(x, (H * 2, W * 2), mode="nearest")
            return self.Conv_0(h) if self.with_conv else h
        if not self.with_conv:
            return up_or_down_sampling.upsample_2d(x, self.fir_kernel, factor=2)
        return self.Conv2d_0(x)


class Downsample(nn.Module):
    """/2 downsampling: strided conv / avg-pool or FIR(+fused conv) (reference :129-163)."""

    def __init__(self, in_ch=None, out_ch=None, with_conv=False, fir=False,
                 fir_kernel=(1, 3, 3, 1)):
        super().__init__()
        out_ch = out_ch if out_ch else in_ch
        if not fir:
            if with_conv:
                self.Conv_0 = conv3x3(in_ch, out_ch, stride=2, padding=0)
        elif with_conv:
            self.Conv2d_0 = up_or_down_sampling.Conv2d(in_ch, out_ch, kernel=3, down=True,
                                                       resample_kernel=fir_kernel, use_bias=True,
                                                       kernel_init=default_init())
        self.fir, self.with_conv = fir, with_conv
        self.fir_kernel = fir_kernel
        self.out_ch = out_ch

    def forward(self, x):
        if not self.fir:
            if self.with_conv:
                return self.Conv_0(F.pad(x, (0, 1, 0, 1)))
            return F.avg_pool2d(x, 2, stride=2)
        if not self.with_conv:
            return up_or_down_sampling.downsample_2d(x, self.fir_kernel, factor=2)
        return self.Conv2d_0(x)


class ResnetBlockDDPMpp(nn.Module):
    """DDPM++ residual block (reference :166-209)."""

    def __init__(self, act, in_ch, out_ch=None, temb_dim=None, conv_shortcut=False,
                 dropout=0.1, skip_rescale=False, init_scale=0.):
        super().__init__()
        out_ch = out_ch if out_ch else in_ch
        self.GroupNorm_0 = nn.GroupNorm(num_groups=min(in_ch // 4, 32), num_channels=in_ch, eps=1e-6)
        self.Conv_0 = conv3x3(in_ch, out_ch)
        if temb_dim is not None:
            self.Dense_0 = nn.Linear(temb_dim, out_ch)
            self.Dense_0.weight.data = default_init()(self.Dense_0.weight.data.shape)
            nn.init.zeros_(self.Dense_0.bias)
        self.GroupNorm_1 = nn.GroupNorm(num_groups=min(out_ch // 4, 32), num_channels=out_ch,
                                        eps=1e-6)
        self.Dropout_0 = nn.Dropout(dropout)
        self.Conv_1 = conv3x3(out_ch, out_ch, init_scale=init_scale)
        if in_ch != out_ch:
            if conv_shortcut:
                self.Conv_2 = conv3x3(in_ch, out_ch)
            else:
                self.NIN_0 = NIN(in_ch, out_ch)
        self.skip_rescale = skip_rescale
        self.act = act
        self.out_ch = out_ch
        self.conv_shortcut = conv_shortcut

    def forward(self, x, temb=None):
        h, x = layers.gn_act_fanout(x, self.GroupNorm_0, self.act)
        h = conv_nobias(h, self.Conv_0)
        bias_nc = self.Conv_0.bias[None, :].expand(x.shape[0], -1)
        if temb is not None:
            bias_nc = bias_nc + layers.temb_proj(self.Dense_0, self.act, temb)
        h = gn_act(h, self.GroupNorm_1, self.act, bias_nc)
        h = self.Dropout_0(h)
        if x.shape[1] != self.out_ch:
            x = self.Conv_2(x) if self.conv_shortcut else self.NIN_0(x)
        return layers.conv_residual(h, self.Conv_1, self.Conv_1.bias, x,
                                    np.sqrt(2.) if self.skip_rescale else 1.0)


class ResnetBlockBigGANpp(nn.Module):
    """BigGAN residual block with optional FIR up/down (reference :212-274)."""

    def __init__(self, act, in_ch, out_ch=None, temb_dim=None, up=False, down=False,
                 dropout=0.1, fir=False, fir_kernel=(1, 3, 3, 1), skip_rescale=True,
                 init_scale=0.):
        super().__init__()
        out_ch = out_ch if out_ch else in_ch
        self.GroupNorm_0 = nn.GroupNorm(num_groups=min(in_ch // 4, 32), num_channels=in_ch, eps=1e-6)
        self.up, self.down = up, down
        self.fir, self.fir_kernel = fir, fir_kernel
        self.Conv_0 = conv3x3(in_ch, out_ch)
        if temb_dim is not None:
            self.Dense_0 = nn.Linear(temb_dim, out_ch)
            self.Dense_0.weight.data = default_init()(self.Dense_0.weight.shape)
            nn.init.zeros_(self.Dense_0.bias)
        self.GroupNorm_1 = nn.GroupNorm(num_groups=min(out_ch // 4, 32), num_channels=out_ch,
                                        eps=1e-6)
        self.Dropout_0 = nn.Dropout(dropout)
        self.Conv_1 = conv3x3(out_ch, out_ch, init_scale=init_scale)
        if in_ch != out_ch or up or down:
            self.Conv_2 = conv1x1(in_ch, out_ch)
        self.skip_rescale = skip_rescale
        self.act = act
        self.in_ch, self.out_ch = in_ch, out_ch

    def _resample(self, t):
        if self.up:
            return (up_or_down_sampling.upsample_2d(t, self.fir_kernel, factor=2) if self.fir
                    else up_or_down_sampling.naive_upsample_2d(t, factor=2))
        if self.down:
            return (up_or_down_sampling.downsample_2d(t, self.fir_kernel, factor=2) if self.fir
                    else up_or_down_sampling.naive_downsample_2d(t, factor=2))
        return t

    def forward_pair(self, x1, x2, temb=None):
        """forward(torch.cat([x1, x2], 1), temb) -- the up path's skip concatenation -- at
        inference without building the concatenation: GroupNorm_0 from the parts' partial
        statistics, Conv_0 reading both sources (Winograd), the 1x1 skip projection as one
        two-source MFMA GEMM.  Falls back to the concatenation when a piece does not fit."""
        from op import conv as conv_op
        from op.norm_act import group_norm_affine_partials
        C1, C = x1.shape[1], x1.shape[1] + x2.shape[1]
        ok = (layers.fused_inference_ok(self, x1, self.act) and not (self.up or self.down)
              and hasattr(self, "Conv_2") and C1 % 8 == 0
              and x1.dtype == torch.float32 and self.Conv_0.weight.shape[1] == C
              and bool(conv_op.lib.bpk_conv3x3_wino_supported(
                  x1.shape[0], C, self.Conv_0.out_channels, x1.shape[2], x1.shape[3]))
              and conv_op.gemm1x1_supported(x1, self.Conv_2.weight, x2))
        if ok:
            # partial statistics of both parts (one read of a part whose producer wrote
            # none: still cheaper than concatenating and reading the concatenation)
            p1, p2 = conv_op.ensure_gn_partials(x1), conv_op.ensure_gn_partials(x2)
            ok = p1 is not None and p2 is not None and p1[1:] == p2[1:]
        if not ok:
            return self.forward(layers.cat_channels(x1, x2), temb)
        ss = group_norm_affine_partials(p1, x1.shape[0], C, self.GroupNorm_0, part2=p2)
        h = conv_op.conv3x3_pair(x1, x2, self.Conv_0.weight, pre=ss,
                                 stats=layers._GN_STATS)
        bias_nc = self.Conv_0.bias[None, :].expand(h.shape[0], -1)
        if temb is not None:
            bias_nc = bias_nc + layers.temb_proj(self.Dense_0, self.act, temb)
        bias = self.Conv_1.bias + self.Conv_2.bias
        x = conv_op.conv1x1(x1, self.Conv_2.weight, None, x2)
        div = np.sqrt(2.) if self.skip_rescale else 1.0
        out = layers.gn_silu_conv(h, self.GroupNorm_1, self.Conv_1, bias_nc, bias, x, div)
        if out is not None:
            return out
        h = gn_act(h, self.GroupNorm_1, self.act, bias_nc)
        return layers.conv_residual(h, self.Conv_1, bias, x, div, stats=True)

    def forward(self, x, temb=None):
        fused = layers.fused_inference_ok(self, x, self.act)
        h = None
        if fused and not (self.up or self.down):
            # GroupNorm_0 + SiLU applied inside Conv_0's input load (inference)
            h = layers.gn_silu_conv(x, self.GroupNorm_0, self.Conv_0)
        link = None
        if h is None and not (self.up or self.down):
            # eval-mode autograd (DPS): the same fusion, its backward recomputing the normalization
            link = layers.skip_link(self, self.in_ch == self.out_ch
                                    and layers._dropout_off(self.Dropout_0))
            r = layers.gn_silu_conv_ad(self, x, self.GroupNorm_0, self.Conv_0, self.act,
                                       take=link, fanout=self.in_ch != self.out_ch)
            h = None
            if r is None:
                link = None
            else:
                h, x = r
        if h is None:
            h, x = layers.gn_act_fanout(x, self.GroupNorm_0, self.act)
            h = self._resample(h)
            x = self._resample(x)
            h = conv_nobias(h, self.Conv_0)
        bias_nc = self.Conv_0.bias[None, :].expand(h.shape[0], -1)
        if temb is not None:
            bias_nc = bias_nc + layers.temb_proj(self.Dense_0, self.act, temb)
        bias = self.Conv_1.bias
        if self.in_ch != self.out_ch or self.up or self.down:
            # the 1x1 skip conv's bias joins Conv_1's in the fused residual (no separate
            # full-tensor bias add after the GEMM)
            x = conv_nobias(x, self.Conv_2)
            bias = bias + self.Conv_2.bias
        div = np.sqrt(2.) if self.skip_rescale else 1.0
        if fused:
            # GroupNorm_1 (+ time bias) + SiLU + Conv_1 + residual tail: two launches
            out = layers.gn_silu_conv(h, self.GroupNorm_1, self.Conv_1, bias_nc, bias, x, div)
            if out is not None:
                return out
        elif layers._dropout_off(self.Dropout_0):
            out = layers.gn_silu_conv_ad_1(self, h, self.GroupNorm_1, self.Conv_1, self.act,
                                           bias_nc=bias_nc, conv_bias=bias, skip=x, div=div,
                                           give=link)
            if out is not None:
                return out
        h = gn_act(h, self.GroupNorm_1, self.act, bias_nc)
        h = self.Dropout_0(h)
        return layers.conv_residual(h, self.Conv_1, bias, x, div, stats=fused)
