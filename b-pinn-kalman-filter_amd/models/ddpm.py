"""DDPM U-Net (the fork's "DDPM++" configs use it), `@register_model('ddpm')`.

Reference: models/ddpm.py:39-183 (+ `UNet = DDPM`, :183).  Module order (and
therefore state-dict keys) matches the reference; forward runs a precomputed
plan like NCSN++ (models/ncsnpp.py in this package).
"""
from __future__ import annotations

import functools

import torch
import torch.nn as nn

from . import layers, utils

conv3x3 = layers.ddpm_conv3x3
default_initializer = layers.default_init


@utils.register_model(name="ddpm")
class DDPM(nn.Module):
    def __init__(self, config):
        super().__init__()
        m = config.model
        self.act = act = layers.get_act(config)
        self.register_buffer("sigmas", torch.tensor(utils.get_sigmas(config)))
        self.nf = nf = m.nf
        ch_mult = m.ch_mult
        self.num_res_blocks = nrb = m.num_res_blocks
        self.attn_resolutions = attn_res = m.attn_resolutions
        self.num_resolutions = nres = len(ch_mult)
        self.all_resolutions = res_at = [config.data.image_size // (2 ** i) for i in range(nres)]
        self.conditional = m.conditional
        self.centered = config.data.centered
        self.scale_by_sigma = m.scale_by_sigma
        channels = config.data.num_channels
        Res = functools.partial(layers.ResnetBlockDDPM, act=act, temb_dim=4 * nf, dropout=m.dropout)

        mods: list = []
        plan: list = []

        def add(module, *step):
            mods.append(module)
            if step:
                plan.append((step[0], len(mods) - 1) + tuple(step[1:]))

        if self.conditional:
            for fan_in in (nf, nf * 4):
                lin = nn.Linear(fan_in, nf * 4)
                lin.weight.data = default_initializer()(lin.weight.data.shape)
                nn.init.zeros_(lin.bias)
                add(lin)
        # NOTE: the reference only defines `modules` inside `if conditional`
        # (models/ddpm.py:57-63), so unconditional DDPM raises there.
        add(conv3x3(channels, nf), "conv_in")
        hs_c = [nf]
        in_ch = nf
        for lvl in range(nres):
            for _ in range(nrb):
                out_ch = nf * ch_mult[lvl]
                add(Res(in_ch=in_ch, out_ch=out_ch), "res", "top")
                in_ch = out_ch
                if res_at[lvl] in attn_res:
                    add(layers.AttnBlock(channels=in_ch), "attn")
                hs_c.append(in_ch)
                plan.append(("push",))
            if lvl != nres - 1:
                add(layers.Downsample(channels=in_ch, with_conv=m.resamp_with_conv), "down_push")
                hs_c.append(in_ch)
        in_ch = hs_c[-1]
        plan.append(("h_from_top",))
        add(Res(in_ch=in_ch), "res", "h")
        add(layers.AttnBlock(channels=in_ch), "attn")
        add(Res(in_ch=in_ch), "res", "h")
        for lvl in reversed(range(nres)):
            for _ in range(nrb + 1):
                out_ch = nf * ch_mult[lvl]
                add(Res(in_ch=in_ch + hs_c.pop(), out_ch=out_ch), "res_cat")
                in_ch = out_ch
            if res_at[lvl] in attn_res:
                add(layers.AttnBlock(channels=in_ch), "attn")
            if lvl != 0:
                add(layers.Upsample(channels=in_ch, with_conv=m.resamp_with_conv), "up")
        assert not hs_c
        gi = len(mods)
        mods.append(nn.GroupNorm(num_channels=in_ch, num_groups=32, eps=1e-6))
        mods.append(conv3x3(in_ch, channels, init_scale=0.))
        plan.append(("head", gi, gi + 1))
        self.all_modules = nn.ModuleList(mods)
        self._plan = plan

    def forward(self, x, labels):
        mods = self.all_modules
        if self.conditional:
            temb = layers.get_timestep_embedding(labels, self.nf)
            temb = layers.dense(mods[0], temb)
            temb = layers.dense(mods[1], self.act(temb))
        else:
            temb = None
        fused = layers._DDPM_FUSED and layers.fused_inference_ok(self, x, self.act)
        if temb is not None and x.is_cuda and (fused or layers._TEMB_BANK_AD):
            # every block's Dense_0 projection of act(temb) as one GEMM (layers.TembBank)
            temb = layers.TembBank(temb, self.act, [m.Dense_0 for m in mods
                                                    if isinstance(m, layers.ResnetBlockDDPM)])
        h = x if self.centered else 2 * x - 1.
        x_in = h
        hs: list = []
        for step in self._plan:
            kind = step[0]
            if kind == "conv_in":
                h = mods[step[1]](x_in)
                hs.append(h)
            elif kind == "res":
                h = mods[step[1]](hs[-1] if step[2] == "top" else h, temb)
            elif kind == "attn":
                h = mods[step[1]](h)
            elif kind == "push":
                hs.append(h)
            elif kind == "down_push":
                hs.append(mods[step[1]](hs[-1]))
            elif kind == "h_from_top":
                h = hs[-1]
            elif kind == "res_cat":
                h = mods[step[1]].forward_pair(h, hs.pop(), temb)
            elif kind == "up":
                h = mods[step[1]](h)
            elif kind == "head":
                y = None
                if fused:  # GroupNorm+SiLU in the output conv's input load
                    y = layers.gn_silu_conv(h, mods[step[1]], mods[step[2]],
                                            conv_bias=mods[step[2]].bias)
                h = y if y is not None else mods[step[2]](layers.gn_act(h, mods[step[1]], self.act))
        assert not hs
        if self.scale_by_sigma:
            h = h / self.sigmas[labels, None, None, None]
        return h


UNet = DDPM
