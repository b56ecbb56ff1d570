"""Shared score-network layers on the gfx950 path (reference: models/layers.py).

Parameter names and initialisation follow the reference so that state dicts
(and therefore reference checkpoints) load unchanged; the arithmetic runs on
the fused HIP ops of `op.norm_act` (GroupNorm + bias + SiLU, residual rescale).
"""
from __future__ import annotations

import contextlib
import math
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from op import channels
from op import conv as conv_op
from op import matmul as matmul_op
from op import norm_act as norm_act_op
from op.norm_act import ACT_NONE, ACT_SILU, group_norm_act, group_norm_affine, residual_rescale


def get_act(config):
    """Activation module from config.model.nonlinearity (reference layers.py:29-41)."""
    name = config.model.nonlinearity.lower()
    table = {"elu": nn.ELU, "relu": nn.ReLU, "swish": nn.SiLU}
    if name == "lrelu":
        return nn.LeakyReLU(negative_slope=0.2)
    if name not in table:
        raise NotImplementedError("activation function does not exist!")
    return table[name]()


def dense(m: nn.Linear, x):
    """m(x) for an nn.Linear: the native GEMM on HIP tensors (op.matmul.linear, forward and
    gradients), nn.Linear itself elsewhere."""
    if x.is_cuda and matmul_op.supported(x, m.weight, m.bias):
        return matmul_op.linear(x, m.weight, m.bias)
    return m(x)


# the bank under autograd too (training, DPS); A/B switch
_TEMB_BANK_AD = os.environ.get("BPK_TEMB_BANK_AD", "1") == "1"


class TembBank:
    """act(temb) projected by every residual block's Dense_0 at once: one concatenation of the
    weights and one GEMM per forward instead of ~34 latency-bound [B, 4 nf] x [4 nf, C] Linear
    launches (and one SiLU instead of one per block).  Under autograd the backward is then
    one GEMM per gradient too (the weight gradients of all blocks in one launch, split back
    into each Dense_0's as views), instead of three launches and an add per block.  Built per
    forward from the live weights (no cache to go stale when EMA / load_state_dict / an
    optimizer step rewrite them).  The same values as per-block Linear calls: each output is
    the same dot product over the same K order."""

    def __init__(self, temb, act, denses):
        self._idx = {}
        sizes = []
        for i, d in enumerate(denses):
            self._idx[id(d)] = i
            sizes.append(d.out_features)
        w = channels.cat([d.weight for d in denses], 0)
        b = channels.cat([d.bias for d in denses], 0)
        a = act(temb)
        allp = (matmul_op.linear(a, w, b) if a.is_cuda and matmul_op.supported(a, w, b)
                else torch.addmm(b, a, w.t()))
        # per-block views; under autograd one split (its backward: one concatenation) rather
        # than a slice per block (a zero-filled full-size gradient per slice, then the adds)
        self.parts = channels.split(allp, sizes, 1)

    def proj(self, dense):
        return self.parts[self._idx[id(dense)]]


def temb_proj(dense_m: nn.Linear, act, temb):
    """dense(act(temb)) -- a TembBank slice when the forward built one."""
    if isinstance(temb, TembBank):
        return temb.proj(dense_m)
    return dense(dense_m, act(temb))


_GN_FANOUT = os.environ.get("BPK_GN_FANOUT", "1") == "1"  # A/B switch (gn_act_fanout)


def gn_act_fanout(x, gn: nn.GroupNorm, act=None):
    """(gn_act(x, gn, act), x) for a residual block whose input also feeds its skip: under
    autograd the skip's gradient is added inside the GroupNorm backward kernel
    (op.norm_act.group_norm_act_fanout) instead of by a separate accumulation launch."""
    if (_GN_FANOUT and torch.is_grad_enabled() and x.requires_grad and x.is_cuda
            and x.dtype == torch.float32 and (act is None or isinstance(act, nn.SiLU))):
        from op.norm_act import group_norm_act_fanout
        return group_norm_act_fanout(x, gn, ACT_NONE if act is None else ACT_SILU)
    return gn_act(x, gn, act), x


def gn_act(x, gn: nn.GroupNorm, act=None, bias_nc=None):
    """act(GroupNorm(x + bias_nc)); SiLU (and no activation) fuse into one HIP launch."""
    if act is None:
        return group_norm_act(x, gn, ACT_NONE, bias_nc)
    if isinstance(act, nn.SiLU):
        return group_norm_act(x, gn, ACT_SILU, bias_nc)
    return act(group_norm_act(x, gn, ACT_NONE, bias_nc))


def variance_scaling(scale, mode, distribution, in_axis=1, out_axis=0, dtype=torch.float32,
                     device="cpu"):
    """JAX-style variance-scaling initializer (reference layers.py:54-80)."""

    def init(shape, dtype=dtype, device=device):
        receptive = np.prod(shape) / shape[in_axis] / shape[out_axis]
        fan_in = shape[in_axis] * receptive
        fan_out = shape[out_axis] * receptive
        denom = {"fan_in": fan_in, "fan_out": fan_out, "fan_avg": (fan_in + fan_out) / 2}.get(mode)
        if denom is None:
            raise ValueError(f"invalid mode for variance scaling initializer: {mode}")
        variance = scale / denom
        if distribution == "normal":
            return torch.randn(*shape, dtype=dtype, device=device) * np.sqrt(variance)
        if distribution == "uniform":
            return (torch.rand(*shape, dtype=dtype, device=device) * 2. - 1.) * np.sqrt(3 * variance)
        raise ValueError("invalid distribution for variance scaling initializer")

    return init


def default_init(scale=1.):
    """DDPM initialisation (reference layers.py:83-86)."""
    return variance_scaling(1e-10 if scale == 0 else scale, "fan_avg", "uniform")


def ddpm_conv1x1(in_planes, out_planes, stride=1, bias=True, init_scale=1., padding=0):
    conv = nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, padding=padding, bias=bias)
    conv.weight.data = default_init(init_scale)(conv.weight.data.shape)
    if bias:
        nn.init.zeros_(conv.bias)
    return conv


# Fusion switches: module constants (each measured against the unfused form, DESIGN.md
# section 4); tests flip them to compare against the unfused composition.
_WINO_ENABLED = True  # 3x3 convs on the Winograd kernels (False: MIOpen)
_IN_FUSED = True      # InstanceNorm+ELU (+ backward, double backward) as one kernel each
_GN_STATS = True      # GroupNorm partial statistics from the producing conv's epilogue
_GEMM1X1 = True       # 1x1 convs on the MFMA GEMM kernels
_DDPM_FUSED = True    # ResnetBlockDDPM inference on the GroupNorm-prologue Winograd convs
# eval-mode autograd (DPS): GroupNorm+SiLU inside the conv's input load.  Its backward is
# first-order only (once_differentiable): create_graph=True / higher derivatives through an
# eval-mode score net need BPK_GN_CONV_AD=0 or the `higher_order_autograd()` block below
_GN_CONV_AD = os.environ.get("BPK_GN_CONV_AD", "1") == "1"
# the same under training (A/B switch, BPK_GN_CONV_AD_TRAIN=1)
_GN_CONV_AD_TRAIN = os.environ.get("BPK_GN_CONV_AD_TRAIN", "0") == "1"


def _is_3x3(x, conv: nn.Conv2d):
    return (_WINO_ENABLED and conv.kernel_size == (3, 3) and conv.stride == (1, 1)
            and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1
            and x.is_cuda and x.dtype == torch.float32 and conv.weight.dtype == torch.float32)


def _is_1x1(x, conv: nn.Conv2d):
    return (_WINO_ENABLED and _GEMM1X1 and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.padding == (0, 0) and conv.groups == 1 and x.is_cuda)


def _wino_eligible(x, conv: nn.Conv2d):
    """a 3x3 conv one of the native kernels (Winograd MFMA, small-channel) runs"""
    return _is_3x3(x, conv) and conv_op.supported(x, conv.weight)


def conv2d(x, conv: nn.Conv2d, bias=True):
    """conv(x) -- the fused Winograd F(2x2,3x3) MFMA kernel (op.conv) for every 3x3 /
    stride-1 / pad-1 conv whose shape it supports, MIOpen (F.conv2d) otherwise."""
    b = conv.bias if bias else None
    if _is_3x3(x, conv):  # native kernels where they fit; every derivative order on 3x3 ops
        return conv_op.conv3x3(x, conv.weight, b)
    if _is_1x1(x, conv) and conv_op.conv1x1_train_supported(x, conv.weight):
        return conv_op.conv1x1_ad(x, conv.weight, b)  # MFMA GEMMs, every derivative order
    if (x.is_cuda and _WINO_ENABLED and conv.padding_mode == "zeros"
            and isinstance(conv.padding, tuple)):
        # implicit-GEMM MFMA kernels; under autograd every derivative order stays a plain
        # convolution (op.conv.conv2d_general)
        return conv_op.conv2d_general(x, conv.weight, b, conv.stride, conv.padding,
                                      conv.dilation, conv.groups)
    return F.conv2d(x, conv.weight, b, conv.stride, conv.padding, conv.dilation, conv.groups)


def fused_inference_ok(module: nn.Module, x, act) -> bool:
    """True when a block may take the inference-only fused paths (GroupNorm + SiLU applied
    inside the Winograd conv's input load): eval mode (dropout is the identity), SiLU, and no
    autograd graph to record."""
    if module.training or not isinstance(act, nn.SiLU) or not _WINO_ENABLED:
        return False
    return not (torch.is_grad_enabled() and (x.requires_grad or any(
        p.requires_grad for p in module.parameters())))


def gn_silu_conv(x, gn: nn.GroupNorm, conv: nn.Conv2d, bias_nc=None, conv_bias=None,
                 skip=None, div=1.0):
    """conv(SiLU(GroupNorm(x + bias_nc))) [+ residual tail] in two launches -- the GroupNorm
    statistics pass and the Winograd conv whose patch load applies the normalization -- or
    None when the conv does not qualify."""
    if not _wino_eligible(x, conv) or (skip is not None and skip.shape[1] != conv.out_channels):
        return None
    if conv_op.small_supported(x, conv.weight) and conv.out_channels > 4:
        return None  # the small-Cin kernel has no GroupNorm prologue
    ss = group_norm_affine(x, gn, bias_nc)
    return conv_op.conv3x3(x, conv.weight, conv_bias, skip=skip, div=div, pre=ss,
                           stats=_GN_STATS and conv_op.wino_supported(x, conv.weight))


def gn_silu_conv_ad(module: nn.Module, x, gn: nn.GroupNorm, conv: nn.Conv2d, act, bias_nc=None,
                    conv_bias=None, skip=None, div=1.0, give=None, take=None, fanout=False):
    """gn_silu_conv under autograd for an eval-mode block (DPS: gradients of the score w.r.t.
    the input through the net): conv(SiLU(GroupNorm(x + bias_nc))) [+ residual tail] with the
    normalization inside the Winograd conv's input load and a backward that recomputes it
    (op.conv.gn_silu_conv3x3_ad); None when it does not apply (training, no autograd graph to
    record, another activation, a conv the kernel does not take).  Training keeps the unfused
    composition: on the DSM and CIFAR train steps the fused form measured 2.8 % and 1.5 %
    slower (the weight gradient's per-element SiLU in its patch load, the igemm choice lost
    on small images), DPS 4.1 % faster (profiles/r05_gn_conv_ad_ab.txt).
    Returns (output, x') or None; x' is x itself, or with fanout=True (a block whose shortcut
    conv reads x) x through the fused Function, so the shortcut's gradient joins the GroupNorm
    backward's pass instead of an accumulation launch."""
    if not (_GN_CONV_AD and (not module.training or _GN_CONV_AD_TRAIN) and torch.is_grad_enabled()
            and isinstance(act, nn.SiLU) and _is_3x3(x, conv)):
        return None
    if skip is not None and skip.shape[1] != conv.out_channels:
        return None
    fanout = fanout and _GN_FANOUT and x.requires_grad
    r = conv_op.gn_silu_conv3x3_ad(x, gn.num_groups, gn.weight if gn.affine else None,
                                   gn.bias if gn.affine else None, gn.eps, conv.weight,
                                   conv_bias, skip, div, bias_nc, give, take, fanout)
    if r is None or not fanout:
        return r if r is None else (r, x)
    return r


def gn_silu_conv_ad_1(module: nn.Module, x, gn: nn.GroupNorm, conv: nn.Conv2d, act, **kw):
    """gn_silu_conv_ad's output alone (or None)"""
    r = gn_silu_conv_ad(module, x, gn, conv, act, **kw)
    return None if r is None else r[0]


@contextlib.contextmanager
def higher_order_autograd():
    """Inside this block eval-mode blocks record the unfused composition (every op
    differentiable to any order) instead of the first-order-only fused GroupNorm+SiLU conv, skip
    link and GroupNorm fan-out: for create_graph=True / double backward through a score net (the DPS and
    likelihood paths of the reference are first-order and do not need it)."""
    global _GN_CONV_AD, _SKIP_LINK, _GN_FANOUT
    prev = _GN_CONV_AD, _SKIP_LINK, _GN_FANOUT
    _GN_CONV_AD, _SKIP_LINK, _GN_FANOUT = False, False, False
    try:
        yield
    finally:
        _GN_CONV_AD, _SKIP_LINK, _GN_FANOUT = prev


def skip_link(module: nn.Module, identity_skip: bool):
    """A conv_op.SkipLink for a residual block whose skip is its input itself, when the block
    is about to take the fused autograd path for both convs: the second conv then hands its
    skip gradient to the first conv's GroupNorm backward (no separate accumulation launch)."""
    return conv_op.SkipLink() if (_SKIP_LINK and identity_skip and not module.training
                                  and torch.is_grad_enabled()) else None


_SKIP_LINK = os.environ.get("BPK_SKIP_LINK", "1") == "1"  # A/B switch
# ResidualBlock (PressureNet): the input's two gradients added in the norm's backward kernel
_IN_FANOUT = os.environ.get("BPK_IN_FANOUT", "1") == "1"


def _dropout_off(m: nn.Dropout) -> bool:
    return not m.training or m.p == 0


def conv_residual(h, conv: nn.Conv2d, bias, skip, div, stats=False):
    """(skip + (conv(h) + bias)) / div -- the tail of every residual block -- as ONE
    Winograd launch when the conv qualifies, else conv + the fused residual kernel.
    stats=True (inference): the output carries GroupNorm partial statistics."""
    if _wino_eligible(h, conv) and skip.shape[1] == conv.out_channels:
        return conv_op.conv3x3(h, conv.weight, bias, skip=skip, div=div,
                               stats=_GN_STATS and stats and conv_op.wino_supported(h, conv.weight))
    return residual_rescale(skip, conv2d(h, conv, bias=False), bias, div)


def cat_channels(a, b):
    """torch.cat([a, b], 1); GroupNorm partial statistics carried by both inputs are
    concatenated too (per-channel partials over the same regions)."""
    y = torch.cat([a, b], dim=1)
    pa, pb = conv_op.gn_partials(a), conv_op.gn_partials(b)
    if pa is not None and pb is not None and pa[1:] == pb[1:]:
        conv_op.attach_gn_partials(y, torch.cat([pa[0], pb[0]], dim=1), pa[1], pa[2])
    return y


class Conv2d(nn.Conv2d):
    """nn.Conv2d (same parameters / state-dict keys) whose forward is `conv2d` above."""

    def forward(self, x):
        return conv2d(x, self)


class ConvTranspose2d(nn.ConvTranspose2d):
    """nn.ConvTranspose2d (same parameters / state-dict keys) as the adjoint of a conv on the
    implicit-GEMM MFMA kernels, every derivative order a plain convolution
    (op.conv.conv_transpose2d_general)."""

    def forward(self, x, output_size=None):
        if (not x.is_cuda or not _WINO_ENABLED or output_size is not None
                or self.padding_mode != "zeros" or isinstance(self.padding, str)):
            return super().forward(x, output_size)
        return conv_op.conv_transpose2d_general(x, self.weight, self.bias, self.stride,
                                                self.padding, self.output_padding, self.groups,
                                                self.dilation)


def ddpm_conv3x3(in_planes, out_planes, stride=1, bias=True, dilation=1, init_scale=1., padding=1):
    conv = Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=padding,
                  dilation=dilation, bias=bias)
    conv.weight.data = default_init(init_scale)(conv.weight.data.shape)
    if bias:
        nn.init.zeros_(conv.bias)
    return conv


def conv_nobias(x, conv: nn.Conv2d):
    """Run a Conv2d module without its bias (the bias is folded into a later fused op)."""
    return conv2d(x, conv, bias=False)


_FREQS: dict = {}


def _freqs(half, max_positions, device):
    """exp(arange(half) * -log(max_positions) / (half - 1)) as the reference computes it, once per
    (half, device): a constant of the net (three launches per call otherwise, recorded into the
    PINN step's graph at every level)."""
    key = (half, max_positions, str(device))
    f = _FREQS.get(key)
    if f is None:
        rate = math.log(max_positions) / (half - 1)
        f = torch.exp(torch.arange(half, dtype=torch.float32, device=device) * -rate)
        _FREQS[key] = f
    return f


def get_timestep_embedding(timesteps, embedding_dim, max_positions=10000):
    """Sinusoidal embedding (reference layers.py:500-514)."""
    assert timesteps.ndim == 1
    half = embedding_dim // 2
    freqs = _freqs(half, max_positions, timesteps.device)
    arg = timesteps.float()[:, None] * freqs[None, :]
    emb = channels.cat([torch.sin(arg), torch.cos(arg)], dim=1)  # = torch.cat, any derivative order
    if embedding_dim % 2 == 1:
        emb = F.pad(emb, (0, 1), mode="constant")
    return emb


_SPATIAL_GROUPS = 1  # batch = this many independent copies (spatial_groups)


@contextlib.contextmanager
def spatial_groups(k):
    """Inside this block the batch of get_spatial_embedding is k stacked copies of one batch
    (pinn.PINN.forward_residual_copies): x.max() / y.max() -- which couple the samples of a
    batch -- are taken per copy, so every copy computes (and differentiates) exactly what the
    single batch would."""
    global _SPATIAL_GROUPS
    prev, _SPATIAL_GROUPS = _SPATIAL_GROUPS, int(k)
    try:
        yield
    finally:
        _SPATIAL_GROUPS = prev


def _max_minus(v):
    """v.max() - v, the max per copy under spatial_groups(k) (ties share the gradient evenly
    within a copy, as max() does over one batch)."""
    k = _SPATIAL_GROUPS
    if k == 1:
        return v.max() - v
    g = v.reshape((k, v.shape[0] // k) + tuple(v.shape[1:]))
    m = g.reshape(k, -1).amax(1).view((k,) + (1,) * (g.dim() - 1))
    return (m - g).reshape(v.shape)


_SEMB_FUSED = os.environ.get("BPK_SEMB_FUSED", "1") == "1"  # A/B switch
_RES_TAIL = os.environ.get("BPK_RES_TAIL", "1") == "1"  # ResidualBlock: skip add in conv2


def get_timestep_embeddings(timesteps, dims, max_positions=10000):
    """[get_timestep_embedding(timesteps, d) for d in dims] (the same values) with one product,
    one sin and one cos for all of them: FlowNet embeds t at every pyramid level, and the PINN
    residual differentiates each embedding w.r.t. t (u_t, v_t) -- per level a chain of
    launches in every pass, here one."""
    assert timesteps.ndim == 1
    halves = [d // 2 for d in dims]
    parts = [h for h in halves if h > 0]
    out = [None] * len(dims)
    if parts:
        key = ("cat", tuple(parts), max_positions, str(timesteps.device))
        freqs = _FREQS.get(key)
        if freqs is None:
            freqs = torch.cat([_freqs(h, max_positions, timesteps.device) for h in parts])
            _FREQS[key] = freqs
        arg = timesteps.float()[:, None] * freqs[None, :]
        sins = iter(channels.split(torch.sin(arg), parts, 1))
        coss = iter(channels.split(torch.cos(arg), parts, 1))
    for i, (d, h) in enumerate(zip(dims, halves)):
        if h > 0:
            emb = channels.cat([next(sins), next(coss)], dim=1)
        else:
            emb = timesteps.new_zeros((timesteps.shape[0], 0), dtype=torch.float32)
        if d % 2 == 1:
            emb = F.pad(emb, (0, 1), mode="constant")
        out[i] = emb
    return out


def get_spatial_embedding(x, y, omega, s=1.0):
    """Spatial embedding of the PINN nets (reference layers.py:517-521).  On HIP tensors: one
    native op with its first and second derivatives (op.embedding; the same forward bits)."""
    if _SEMB_FUSED and x.is_cuda:
        from op import embedding
        if embedding.supported(x, y, _SPATIAL_GROUPS):
            return embedding.spatial_embedding(x, y, omega, s, _SPATIAL_GROUPS)
    e1 = torch.sin(omega * torch.sqrt(x ** 2 + y ** 2))
    e2 = torch.sin(omega * torch.sqrt(_max_minus(x) ** 2 + _max_minus(y) ** 2))
    return (e1 + e2) / s


class NIN(nn.Module):
    """Per-pixel dense layer: y[b, :, h, w] = x[b, :, h, w] @ W + b (reference layers.py:537-546)."""

    def __init__(self, in_dim, num_units, init_scale=0.1):
        super().__init__()
        self.W = nn.Parameter(default_init(scale=init_scale)((in_dim, num_units)), requires_grad=True)
        self.b = nn.Parameter(torch.zeros(num_units), requires_grad=True)

    def forward(self, x):
        # 1x1 convolution with weight W^T: the MFMA GEMM kernels (forward and every
        # derivative, op.conv.conv1x1_ad) on HIP tensors
        w = self.W.t()
        if _GEMM1X1 and x.is_cuda and conv_op.conv1x1_train_supported(x, w):
            return conv_op.conv1x1_ad(x, w, self.b)
        if _WINO_ENABLED and x.is_cuda:
            # planes the 1x1 GEMM does not take (H * W % 128: the 4 x 4 attention of the
            # CIFAR-10 net): the implicit-GEMM kernels -- MIOpen ran them on its naive
            # reference kernel, 0.7 ms forward / 1.4 ms backward per call
            return conv_op.conv2d_general(x, w[:, :, None, None], self.b)
        return F.conv2d(x, w[:, :, None, None], self.b)


def _attention(h, nin_q, nin_k, nin_v):
    """softmax(q^T k / sqrt(C)) over the H*W positions, returns [B, C, H, W]."""
    B, C, H, W = h.shape
    q = nin_q(h).reshape(B, C, H * W)
    k = nin_k(h).reshape(B, C, H * W)
    v = nin_v(h).reshape(B, C, H * W)
    mm = matmul_op.bmm_ad if h.is_cuda and matmul_op.supported(h) else torch.bmm
    w = mm(q.transpose(1, 2), k) * (int(C) ** (-0.5))  # [B, HW(q), HW(k)]
    w = torch.softmax(w, dim=-1)
    out = mm(v, w.transpose(1, 2))  # [B, C, HW(q)]
    return out.reshape(B, C, H, W)


class AttnBlock(nn.Module):
    """DDPM channel attention block (reference layers.py:549-573)."""

    def __init__(self, channels, num_groups=32):
        super().__init__()
        self.GroupNorm_0 = nn.GroupNorm(num_groups=num_groups, num_channels=channels, eps=1e-6)
        self.NIN_0 = NIN(channels, channels)
        self.NIN_1 = NIN(channels, channels)
        self.NIN_2 = NIN(channels, channels)
        self.NIN_3 = NIN(channels, channels, init_scale=0.)

    def forward(self, x):
        h = gn_act(x, self.GroupNorm_0, None)
        if _DDPM_FUSED and not torch.is_grad_enabled():
            # inference: AttnBlockpp's stacked q/k/v MFMA GEMM (the same NIN_0..3 layout)
            from .layerspp import _ATTN_QKV, AttnBlockpp
            if _ATTN_QKV and AttnBlockpp._qkv_ok(self, h):
                return residual_rescale(x, AttnBlockpp._forward_qkv(self, h), None, 1.0)
        h = self.NIN_3(_attention(h, self.NIN_0, self.NIN_1, self.NIN_2))
        return residual_rescale(x, h, None, 1.0)


class Upsample(nn.Module):
    """Nearest x2 (+ conv3x3) (reference layers.py:576-590)."""

    def __init__(self, channels, with_conv=False):
        super().__init__()
        if with_conv:
            self.Conv_0 = ddpm_conv3x3(channels, channels)
        self.with_conv = with_conv

    def forward(self, x):
        B, C, H, W = x.shape
        if (self.with_conv and _WINO_ENABLED and x.is_cuda
                and conv_op.up2_supported(x, self.Conv_0.weight)):
            # the upsample read inside the Winograd conv's patch load
            return conv_op.conv3x3_up2(x, self.Conv_0.weight, self.Conv_0.bias)
        h = F.interpolate(x, (H * 2, W * 2), mode="nearest")
        return self.Conv_0(h) if self.with_conv else h


class Downsample(nn.Module):
    """'SAME'-padded strided conv or 2x2 average pool (reference layers.py:593-608)."""

    def __init__(self, channels, with_conv=False):
        super().__init__()
        if with_conv:
            self.Conv_0 = ddpm_conv3x3(channels, channels, stride=2, padding=0)
        self.with_conv = with_conv

    def forward(self, x):
        B, C, H, W = x.shape
        if self.with_conv:
            x = self.Conv_0(F.pad(x, (0, 1, 0, 1)))
        else:
            x = F.avg_pool2d(x, kernel_size=2, stride=2, padding=0)
        assert x.shape == (B, C, H // 2, W // 2)
        return x


class ResnetBlockDDPM(nn.Module):
    """DDPM residual block (reference layers.py:611-655), fused GN+SiLU(+temb bias)."""

    def __init__(self, act, in_ch, out_ch=None, temb_dim=None, conv_shortcut=False, dropout=0.1):
        super().__init__()
        out_ch = out_ch or in_ch
        self.GroupNorm_0 = nn.GroupNorm(num_groups=32, num_channels=in_ch, eps=1e-6)
        self.act = act
        self.Conv_0 = ddpm_conv3x3(in_ch, out_ch)
        if temb_dim is not None:
            self.Dense_0 = nn.Linear(temb_dim, out_ch)
            self.Dense_0.weight.data = default_init()(self.Dense_0.weight.data.shape)
            nn.init.zeros_(self.Dense_0.bias)
        self.GroupNorm_1 = nn.GroupNorm(num_groups=32, num_channels=out_ch, eps=1e-6)
        self.Dropout_0 = nn.Dropout(dropout)
        self.Conv_1 = ddpm_conv3x3(out_ch, out_ch, init_scale=0.)
        if in_ch != out_ch:
            if conv_shortcut:
                self.Conv_2 = ddpm_conv3x3(in_ch, out_ch)
            else:
                self.NIN_0 = NIN(in_ch, out_ch)
        self.out_ch = out_ch
        self.in_ch = in_ch
        self.conv_shortcut = conv_shortcut

    def forward(self, x, temb=None):
        assert x.shape[1] == self.in_ch
        if _DDPM_FUSED and fused_inference_ok(self, x, self.act):
            # inference (the nc_ddpmpp sampler): GroupNorm_0+SiLU inside Conv_0's input load
            h = gn_silu_conv(x, self.GroupNorm_0, self.Conv_0)
            if h is None:
                h = conv_nobias(gn_act(x, self.GroupNorm_0, self.act), self.Conv_0)
            return self._fused_tail(h, x, None, temb)
        link = skip_link(self, self.in_ch == self.out_ch and _dropout_off(self.Dropout_0))
        r = gn_silu_conv_ad(self, x, self.GroupNorm_0, self.Conv_0, self.act, take=link,
                            fanout=self.in_ch != self.out_ch)
        if r is None:
            link = None
            h, x = gn_act_fanout(x, self.GroupNorm_0, self.act)
            h = conv_nobias(h, self.Conv_0)
        else:
            h, x = r
        bias_nc = self.Conv_0.bias[None, :].expand(x.shape[0], -1)
        if temb is not None:
            bias_nc = bias_nc + temb_proj(self.Dense_0, self.act, temb)
        if self.in_ch != self.out_ch:
            x = self.Conv_2(x) if self.conv_shortcut else self.NIN_0(x)
        if _dropout_off(self.Dropout_0):
            out = gn_silu_conv_ad_1(self, h, self.GroupNorm_1, self.Conv_1, self.act,
                                    bias_nc=bias_nc, conv_bias=self.Conv_1.bias, skip=x, div=1.0,
                                    give=link)
            if out is not None:
                return out
        h = gn_act(h, self.GroupNorm_1, self.act, bias_nc)
        h = self.Dropout_0(h)
        return conv_residual(h, self.Conv_1, self.Conv_1.bias, x, 1.0)

    def forward_pair(self, x1, x2, temb=None):
        """forward(torch.cat([x1, x2], 1), temb) -- the up path's skip concatenation -- at
        inference without building it: GroupNorm_0 from both parts' partial statistics,
        Conv_0 reading both sources, NIN_0 as one two-source MFMA GEMM (as
        ResnetBlockBigGANpp.forward_pair); the concatenation when a piece does not fit."""
        N, C1, H, W = x1.shape
        C = C1 + x2.shape[1]
        ok = (_DDPM_FUSED and fused_inference_ok(self, x1, self.act)
              and fused_inference_ok(self, x2, self.act) and C == self.in_ch and C1 % 8 == 0
              and x1.is_cuda and x1.dtype == torch.float32
              and bool(conv_op.lib.bpk_conv3x3_wino_supported(N, C, self.out_ch, H, W)))
        if ok:
            p1, p2 = conv_op.ensure_gn_partials(x1), conv_op.ensure_gn_partials(x2)
            ok = p1 is not None and p2 is not None and p1[1:] == p2[1:]
        if not ok:
            return self.forward(cat_channels(x1, x2), temb)
        ss = norm_act_op.group_norm_affine_partials(p1, N, C, self.GroupNorm_0, part2=p2)
        h = conv_op.conv3x3_pair(x1, x2, self.Conv_0.weight, pre=ss, stats=_GN_STATS)
        return self._fused_tail(h, x1, x2, temb)

    def _fused_tail(self, h, x, x2, temb):
        """(shortcut([x, x2]) + Conv_1(SiLU(GroupNorm_1(h + bias_nc))) + biases) at inference:
        GroupNorm_1+SiLU in Conv_1's input load, the residual in its epilogue, NIN_0's bias
        folded into Conv_1's."""
        bias_nc = self.Conv_0.bias[None, :].expand(h.shape[0], -1)
        if temb is not None:
            bias_nc = bias_nc + temb_proj(self.Dense_0, self.act, temb)
        bias = self.Conv_1.bias
        if self.in_ch == self.out_ch:
            skip = x if x2 is None else cat_channels(x, x2)  # identity of [x, x2]
        elif not self.conv_shortcut and _GEMM1X1 and conv_op.gemm1x1_supported(
                x, self.NIN_0.W.t(), x2):
            skip = conv_op.conv1x1(x, self.NIN_0.W.t(), None, x2)
            bias = bias + self.NIN_0.b
        else:
            xs = x if x2 is None else cat_channels(x, x2)
            skip = self.Conv_2(xs) if self.conv_shortcut else self.NIN_0(xs)
        out = gn_silu_conv(h, self.GroupNorm_1, self.Conv_1, bias_nc, bias, skip, 1.0)
        if out is not None:
            return out
        h = gn_act(h, self.GroupNorm_1, self.act, bias_nc)
        return conv_residual(h, self.Conv_1, bias, skip, 1.0)


# ---------------------------------------------------------------- PINN (NCSN-style) blocks

def ncsn_conv1x1(in_planes, out_planes, stride=1, bias=True, dilation=1, init_scale=1., padding=0):
    """1x1 conv, PyTorch default init scaled by init_scale (reference layers.py:44-50)."""
    conv = Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=bias,
                  dilation=dilation, padding=padding)
    scale = 1e-10 if init_scale == 0 else init_scale
    conv.weight.data *= scale
    if bias:
        conv.bias.data *= scale
    return conv


def ncsn_conv3x3(in_planes, out_planes, stride=1, bias=True, dilation=1, init_scale=1., padding=1):
    """3x3 conv, PyTorch default init scaled by init_scale (reference layers.py:104-110)."""
    scale = 1e-10 if init_scale == 0 else init_scale
    conv = Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, bias=bias,
                  dilation=dilation, padding=padding)
    conv.weight.data *= scale
    if bias:
        conv.bias.data *= scale
    return conv


class ResidualBlock(nn.Module):
    """Pre-activation residual block used by PressureNet (reference layers.py:438-491).

    norm -> act -> conv3x3 -> norm -> act -> conv3x3, plus an identity or 1x1-conv
    shortcut.  Only the `resample=None, dilation=1` form is on the hot path
    (models/flownet.py get_double_res); InstanceNorm2d carries no parameters, so the
    state-dict keys are conv1.*, conv2.* and shortcut.*.  Kept on aten ops: the PINN
    residual differentiates through this block twice (create_graph=True).
    """

    def __init__(self, input_dim, output_dim, resample=None, act=nn.ELU(),
                 normalization=nn.InstanceNorm2d, adjust_padding=False, dilation=1):
        super().__init__()
        if resample is not None or dilation != 1:
            raise NotImplementedError("ResidualBlock: only resample=None, dilation=1 is built")
        self.non_linearity = act
        self.input_dim, self.output_dim = input_dim, output_dim
        self.resample = resample
        self.normalization = normalization
        self.conv1 = ncsn_conv3x3(input_dim, output_dim)
        self.normalize2 = normalization(output_dim)
        self.conv2 = ncsn_conv3x3(output_dim, output_dim)
        if output_dim != input_dim:
            self.shortcut = ncsn_conv1x1(input_dim, output_dim)
        self.normalize1 = normalization(input_dim)

    def _fused_ok(self, norm, x):
        act = self.non_linearity
        return (_IN_FUSED and x.is_cuda and x.dtype in (torch.float32, torch.float64)
                and type(norm) is nn.InstanceNorm2d and not norm.affine
                and not norm.track_running_stats and type(act) is nn.ELU
                and act.alpha == 1.0 and not act.inplace)

    def _norm_act(self, norm, x):
        """act(norm(x)); InstanceNorm2d(affine=False) + ELU(1) on the fused HIP kernels
        (op.norm_act.instance_norm_act: forward, backward and double backward one launch
        each, in place of ~30 aten kernels per norm in the PINN residual's double backward).
        BPK_IN_FUSED=0: aten."""
        act = self.non_linearity
        if (_IN_FUSED and x.is_cuda and x.dtype in (torch.float32, torch.float64)
                and type(norm) is nn.InstanceNorm2d and not norm.affine
                and not norm.track_running_stats and type(act) is nn.ELU
                and act.alpha == 1.0 and not act.inplace):
            return norm_act_op.instance_norm_act(x, norm.eps, norm_act_op.ACT_ELU)
        return act(norm(x))

    def forward(self, x):
        if _IN_FANOUT and self._fused_ok(self.normalize1, x) and torch.is_grad_enabled() \
                and x.requires_grad:
            # x feeds the first norm and the skip: one node takes both gradients and adds them
            # in the norm's backward kernel (op.norm_act.instance_norm_act_fanout)
            a1, xs = norm_act_op.instance_norm_act_fanout(x, self.normalize1.eps,
                                                          norm_act_op.ACT_ELU)
        else:
            a1, xs = self._norm_act(self.normalize1, x), x
        h = self.conv1(a1)
        skip = xs if self.output_dim == self.input_dim else self.shortcut(xs)
        a = self._norm_act(self.normalize2, h)
        if _RES_TAIL and _is_3x3(a, self.conv2):
            # skip + conv2(a) with the add in the conv's epilogue (same rounding: the kernel
            # forms conv + bias, then skip + that); its gradient w.r.t. skip is gy itself
            return conv_op.conv3x3(a, self.conv2.weight, self.conv2.bias, skip=skip)
        return skip + self.conv2(a)
