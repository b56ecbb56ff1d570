"""ORACLE (test infrastructure only) -- score networks restated as pure functions.

`ncsnpp_forward(params, config, x, time_cond)` restates NCSNpp.forward
(reference models/ncsnpp.py:232-381, blocks models/layerspp.py:62-274, FIR
resampling models/up_or_down_sampling.py:144-257) and `ddpm_forward` restates
DDPM.forward (models/ddpm.py:110-181, blocks models/layers.py:537-655), both over
a flat parameter dict keyed exactly like the reference state dict
(`all_modules.{i}.…`).  Torch-CPU float32 ops only.  Pinned by
tests/golden/net_*.npz; also the CPU baseline of bench.py.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from .upfirdn2d_ref import upfirdn2d_torch

_SQRT2 = float(np.sqrt(2.))


def timestep_embedding(t, dim, max_positions=10000):
    """layers.py:500-514."""
    half = dim // 2
    scale = math.log(max_positions) / (half - 1)
    freqs = torch.exp(torch.arange(half, dtype=torch.float32) * -scale)
    arg = t.float()[:, None] * freqs[None]
    out = torch.cat([torch.sin(arg), torch.cos(arg)], 1)
    return F.pad(out, (0, 1)) if dim % 2 else out


def _fir(k, gain):
    k = np.asarray(k, np.float32)
    if k.ndim == 1:
        k = np.outer(k, k)
    k = k / np.sum(k)
    return torch.tensor(k * gain, dtype=torch.float32)


class _P:
    """Cursor over `all_modules.{i}` entries of a state dict."""

    def __init__(self, params):
        self.p = params
        self.i = 0

    def take(self):
        pre = f"all_modules.{self.i}."
        self.i += 1
        return pre

    def __call__(self, key):
        return self.p[key]

    def has(self, key):
        return key in self.p


def _act(name, x):
    name = name.lower()
    if name == "swish":
        return F.silu(x)
    if name == "relu":
        return F.relu(x)
    if name == "elu":
        return F.elu(x)
    if name == "lrelu":
        return F.leaky_relu(x, 0.2)
    raise NotImplementedError(name)


def _gn(P, pre, x, groups=None):
    C = x.shape[1]
    g = groups if groups is not None else min(C // 4, 32)
    return F.group_norm(x, g, P(pre + "weight"), P(pre + "bias"), eps=1e-6)


def _conv(P, pre, x, stride=1, padding=1):
    return F.conv2d(x, P(pre + "weight"), P(pre + "bias") if P.has(pre + "bias") else None,
                    stride=stride, padding=padding)


def _nin(P, pre, x):
    W, b = P(pre + "W"), P(pre + "b")
    y = torch.einsum("bchw,cd->bdhw", x, W)
    return y + b[None, :, None, None]


def _attn(P, pre, x, groups=None, skip_rescale=False):
    """AttnBlockpp (layerspp.py:75-91) / AttnBlock (layers.py:562-573)."""
    B, C, H, W = x.shape
    h = _gn(P, pre + "GroupNorm_0.", x, groups)
    q, k, v = (_nin(P, pre + f"NIN_{j}.", h) for j in range(3))
    w = torch.einsum("bchw,bcij->bhwij", q, k) * (int(C) ** (-0.5))
    w = F.softmax(w.reshape(B, H, W, H * W), dim=-1).reshape(B, H, W, H, W)
    h = torch.einsum("bhwij,bcij->bchw", w, v)
    h = _nin(P, pre + "NIN_3.", h)
    return (x + h) / _SQRT2 if skip_rescale else x + h


def _naive_up(x):
    N, C, H, W = x.shape
    return x.reshape(N, C, H, 1, W, 1).repeat(1, 1, 1, 2, 1, 2).reshape(N, C, 2 * H, 2 * W)


def _naive_down(x):
    N, C, H, W = x.shape
    return x.reshape(N, C, H // 2, 2, W // 2, 2).mean(dim=(3, 5))


def _fir_up(x, k):
    kt = _fir(k, 4)
    p = kt.shape[0] - 2
    return upfirdn2d_torch(x, kt, up=2, pad=((p + 1) // 2 + 1, p // 2))


def _fir_down(x, k):
    kt = _fir(k, 1)
    p = kt.shape[0] - 2
    return upfirdn2d_torch(x, kt, down=2, pad=((p + 1) // 2, p // 2))


def _biggan(P, pre, x, temb, m, up=False, down=False):
    """ResnetBlockBigGANpp (layerspp.py:242-274)."""
    act = m.nonlinearity
    h = _act(act, _gn(P, pre + "GroupNorm_0.", x))
    if up or down:
        if m.fir:
            f = (lambda t: _fir_up(t, m.fir_kernel)) if up else (lambda t: _fir_down(t, m.fir_kernel))
        else:
            f = _naive_up if up else _naive_down
        h, x = f(h), f(x)
    h = _conv(P, pre + "Conv_0.", h)
    if temb is not None:
        h = h + F.linear(_act(act, temb), P(pre + "Dense_0.weight"),
                         P(pre + "Dense_0.bias"))[:, :, None, None]
    h = _act(act, _gn(P, pre + "GroupNorm_1.", h))
    h = _conv(P, pre + "Conv_1.", h)
    if P.has(pre + "Conv_2.weight"):
        x = _conv(P, pre + "Conv_2.", x, padding=0)
    return (x + h) / _SQRT2 if m.skip_rescale else x + h


def _fir_conv_down(P, pre, x, k):
    """Downsample(fir, with_conv) -> Conv2d(down=True) (up_or_down_sampling.py:144-178)."""
    w = P(pre + "Conv2d_0.weight")
    kt = _fir(k, 1)
    p = (kt.shape[0] - 2) + (w.shape[-1] - 1)
    x = upfirdn2d_torch(x, kt, pad=((p + 1) // 2, p // 2))
    x = F.conv2d(x, w, stride=2)
    return x + P(pre + "Conv2d_0.bias").reshape(1, -1, 1, 1)


def ncsnpp_forward(params, config, x, time_cond):
    m = config.model
    P = _P(params)
    nres = len(m.ch_mult)
    res_at = [config.data.image_size // (2 ** i) for i in range(nres)]
    emb = m.embedding_type.lower()
    # time embedding
    if emb == "fourier":
        W = P(P.take() + "W")
        proj = torch.log(time_cond)[:, None] * W[None, :] * 2 * np.pi
        temb = torch.cat([torch.sin(proj), torch.cos(proj)], -1)
        used_sigmas = time_cond
    else:
        temb = timestep_embedding(time_cond, m.nf)
        used_sigmas = None
    if m.conditional:
        pre = P.take()
        temb = F.linear(temb, P(pre + "weight"), P(pre + "bias"))
        pre = P.take()
        temb = F.linear(_act(m.nonlinearity, temb), P(pre + "weight"), P(pre + "bias"))
    else:
        temb = None
    if not config.data.centered:
        x = 2 * x - 1.
    prog_in, prog = m.progressive_input.lower(), m.progressive.lower()
    assert m.resblock_type.lower() == "biggan", "oracle covers the BigGAN block NCSN++"
    pyr_in = x if prog_in != "none" else None
    hs = [_conv(P, P.take(), x)]
    for lvl in range(nres):
        for _ in range(m.num_res_blocks):
            h = _biggan(P, P.take(), hs[-1], temb, m)
            if res_at[lvl] in m.attn_resolutions:
                h = _attn(P, P.take(), h, skip_rescale=m.skip_rescale)
            hs.append(h)
        if lvl != nres - 1:
            h = _biggan(P, P.take(), hs[-1], temb, m, down=True)
            if prog_in == "input_skip":
                pyr_in = _fir_down(pyr_in, m.fir_kernel) if m.fir else F.avg_pool2d(pyr_in, 2, 2)
                pre = P.take()
                hc = _conv(P, pre + "Conv_0.", pyr_in, padding=0)
                h = torch.cat([hc, h], 1) if m.progressive_combine.lower() == "cat" else hc + h
            elif prog_in == "residual":
                pre = P.take()
                if m.fir:
                    pyr_in = _fir_conv_down(P, pre, pyr_in, m.fir_kernel)
                else:
                    pyr_in = _conv(P, pre + "Conv_0.", F.pad(pyr_in, (0, 1, 0, 1)), stride=2,
                                   padding=0)
                pyr_in = (pyr_in + h) / _SQRT2 if m.skip_rescale else pyr_in + h
                h = pyr_in
            hs.append(h)
    h = hs[-1]
    h = _biggan(P, P.take(), h, temb, m)
    h = _attn(P, P.take(), h, skip_rescale=m.skip_rescale)
    h = _biggan(P, P.take(), h, temb, m)
    pyramid = None
    for lvl in reversed(range(nres)):
        for _ in range(m.num_res_blocks + 1):
            h = _biggan(P, P.take(), torch.cat([h, hs.pop()], 1), temb, m)
        if res_at[lvl] in m.attn_resolutions:
            h = _attn(P, P.take(), h, skip_rescale=m.skip_rescale)
        if prog != "none":
            if lvl == nres - 1:
                pg = P.take()
                pc = P.take()
                pyramid = _conv(P, pc, _act(m.nonlinearity, _gn(P, pg, h)))
            elif prog == "output_skip":
                pyramid = _fir_up(pyramid, m.fir_kernel) if m.fir else \
                    F.interpolate(pyramid, scale_factor=2, mode="nearest")
                pg = P.take()
                pc = P.take()
                pyramid = pyramid + _conv(P, pc, _act(m.nonlinearity, _gn(P, pg, h)))
            else:
                raise NotImplementedError("progressive='residual' is unreachable in the reference")
        if lvl != 0:
            h = _biggan(P, P.take(), h, temb, m, up=True)
    assert not hs
    if prog == "output_skip":
        h = pyramid
    else:
        pg = P.take()
        pc = P.take()
        h = _conv(P, pc, _act(m.nonlinearity, _gn(P, pg, h)))
    assert not any(k.startswith(f"all_modules.{P.i}.") for k in params), "unconsumed modules"
    if m.scale_by_sigma:
        if used_sigmas is None:
            used_sigmas = P("sigmas")[time_cond.long()]
        h = h / used_sigmas.reshape((x.shape[0],) + (1,) * (x.ndim - 1))
    return h


def _ddpm_block(P, pre, x, temb, act):
    """ResnetBlockDDPM (layers.py:611-655)."""
    h = _act(act, _gn(P, pre + "GroupNorm_0.", x, 32))
    h = _conv(P, pre + "Conv_0.", h)
    if temb is not None:
        h = h + F.linear(_act(act, temb), P(pre + "Dense_0.weight"),
                         P(pre + "Dense_0.bias"))[:, :, None, None]
    h = _act(act, _gn(P, pre + "GroupNorm_1.", h, 32))
    h = _conv(P, pre + "Conv_1.", h)
    if P.has(pre + "NIN_0.W"):
        x = _nin(P, pre + "NIN_0.", x)
    elif P.has(pre + "Conv_2.weight"):
        x = _conv(P, pre + "Conv_2.", x)
    return x + h


def ddpm_forward(params, config, x, labels):
    m = config.model
    P = _P(params)
    nres = len(m.ch_mult)
    res_at = [config.data.image_size // (2 ** i) for i in range(nres)]
    act = m.nonlinearity
    if m.conditional:
        temb = timestep_embedding(labels, m.nf)
        pre = P.take()
        temb = F.linear(temb, P(pre + "weight"), P(pre + "bias"))
        pre = P.take()
        temb = F.linear(_act(act, temb), P(pre + "weight"), P(pre + "bias"))
    else:
        temb = None
    h = x if config.data.centered else 2 * x - 1.
    hs = [_conv(P, P.take(), h)]
    for lvl in range(nres):
        for _ in range(m.num_res_blocks):
            h = _ddpm_block(P, P.take(), hs[-1], temb, act)
            if res_at[lvl] in m.attn_resolutions:
                h = _attn(P, P.take(), h, groups=32)
            hs.append(h)
        if lvl != nres - 1:
            pre = P.take()
            if m.resamp_with_conv:
                hs.append(_conv(P, pre + "Conv_0.", F.pad(hs[-1], (0, 1, 0, 1)), stride=2,
                                padding=0))
            else:
                hs.append(F.avg_pool2d(hs[-1], 2, 2))
    h = hs[-1]
    h = _ddpm_block(P, P.take(), h, temb, act)
    h = _attn(P, P.take(), h, groups=32)
    h = _ddpm_block(P, P.take(), h, temb, act)
    for lvl in reversed(range(nres)):
        for _ in range(m.num_res_blocks + 1):
            h = _ddpm_block(P, P.take(), torch.cat([h, hs.pop()], 1), temb, act)
        if res_at[lvl] in m.attn_resolutions:
            h = _attn(P, P.take(), h, groups=32)
        if lvl != 0:
            pre = P.take()
            h = F.interpolate(h, scale_factor=2, mode="nearest")
            if m.resamp_with_conv:
                h = _conv(P, pre + "Conv_0.", h)
    assert not hs
    pg = P.take()
    pc = P.take()
    h = _conv(P, pc, _act(act, _gn(P, pg, h, 32)))
    assert not any(k.startswith(f"all_modules.{P.i}.") for k in params), "unconsumed modules"
    if m.scale_by_sigma:
        h = h / P("sigmas")[labels, None, None, None]
    return h


def forward(params, config, x, t):
    if config.model.name == "ncsnpp":
        return ncsnpp_forward(params, config, x, t)
    if config.model.name == "ddpm":
        return ddpm_forward(params, config, x, t)
    raise NotImplementedError(config.model.name)


def init_params(model_state_dict):
    """CPU float32 copy of a state dict (strips a leading 'module.')."""
    out = {}
    for k, v in model_state_dict.items():
        k = k[len("module."):] if k.startswith("module.") else k
        out[k] = v.detach().to("cpu", torch.float32) if v.is_floating_point() else v.cpu()
    return out
