"""NCSN++ score network (reference: models/ncsnpp.py:34-381), `@register_model('ncsnpp')`.

The module list (`all_modules`) is built in the reference's order so state-dict
keys match (`all_modules.{i}.…`).  Alongside it __init__ records a flat
execution plan; forward() interprets the plan instead of re-deriving the
control flow every call, which keeps the per-call Python work small (the PC
sampler calls this 2N times) and makes the whole forward capturable in a
hipGraph.
"""
from __future__ import annotations

import functools

import numpy as np
import torch
import torch.nn as nn

from op.norm_act import residual_rescale

from . import layers, layerspp, utils

# up-path skip concatenations read as two sources at inference (False: torch.cat)
_PAIR = True
# all residual blocks' time-embedding projections as one GEMM at inference
_TEMB_BANK = True
conv3x3 = layerspp.conv3x3
default_initializer = layers.default_init
_SQRT2 = np.sqrt(2.)


@utils.register_model(name="ncsnpp")
class NCSNpp(nn.Module):
    def __init__(self, config):
        super().__init__()
        m = config.model
        self.config = config
        self.act = act = layers.get_act(config)
        self.register_buffer("sigmas", torch.tensor(utils.get_sigmas(config)))
        self.nf = nf = m.nf
        ch_mult = m.ch_mult
        self.num_res_blocks = nrb = m.num_res_blocks
        self.attn_resolutions = attn_res = m.attn_resolutions
        self.num_resolutions = nres = len(ch_mult)
        self.all_resolutions = res_at = [config.data.image_size // (2 ** i) for i in range(nres)]
        self.conditional = m.conditional
        fir, fir_kernel = m.fir, m.fir_kernel
        self.skip_rescale = skip = m.skip_rescale
        self.resblock_type = rtype = m.resblock_type.lower()
        self.progressive = prog = m.progressive.lower()
        self.progressive_input = prog_in = m.progressive_input.lower()
        self.embedding_type = emb = m.embedding_type.lower()
        init_scale = m.init_scale
        assert prog in ["none", "output_skip", "residual"]
        assert prog_in in ["none", "input_skip", "residual"]
        assert emb in ["fourier", "positional"]
        combine = m.progressive_combine.lower()
        channels = config.data.num_channels

        mods: list = []
        plan: list = []

        def add(module, *step):
            mods.append(module)
            if step:
                plan.append((step[0], len(mods) - 1) + tuple(step[1:]))
            return len(mods) - 1

        if emb == "fourier":
            assert config.training.continuous, "Fourier features are only used for continuous training."
            self._temb_idx = add(layerspp.GaussianFourierProjection(embedding_size=nf,
                                                                    scale=m.fourier_scale))
            embed_dim = 2 * nf
        else:
            self._temb_idx = None
            embed_dim = nf
        self._dense_idx = []
        if self.conditional:
            for fan_in in (embed_dim, nf * 4):
                lin = nn.Linear(fan_in, nf * 4)
                lin.weight.data = default_initializer()(lin.weight.shape)
                nn.init.zeros_(lin.bias)
                self._dense_idx.append(add(lin))

        Attn = functools.partial(layerspp.AttnBlockpp, init_scale=init_scale, skip_rescale=skip)
        Up = functools.partial(layerspp.Upsample, with_conv=m.resamp_with_conv, fir=fir,
                               fir_kernel=fir_kernel)
        Down = functools.partial(layerspp.Downsample, with_conv=m.resamp_with_conv, fir=fir,
                                 fir_kernel=fir_kernel)
        if prog == "output_skip":
            self.pyramid_upsample = layerspp.Upsample(fir=fir, fir_kernel=fir_kernel, with_conv=False)
        pyr_up = functools.partial(layerspp.Upsample, fir=fir, fir_kernel=fir_kernel, with_conv=True)
        if prog_in == "input_skip":
            self.pyramid_downsample = layerspp.Downsample(fir=fir, fir_kernel=fir_kernel,
                                                          with_conv=False)
        pyr_down = functools.partial(layerspp.Downsample, fir=fir, fir_kernel=fir_kernel,
                                     with_conv=True)
        if rtype == "ddpm":
            Res = functools.partial(layerspp.ResnetBlockDDPMpp, act=act, dropout=m.dropout,
                                    init_scale=init_scale, skip_rescale=skip, temb_dim=nf * 4)
        elif rtype == "biggan":
            Res = functools.partial(layerspp.ResnetBlockBigGANpp, act=act, dropout=m.dropout,
                                    fir=fir, fir_kernel=fir_kernel, init_scale=init_scale,
                                    skip_rescale=skip, temb_dim=nf * 4)
        else:
            raise ValueError(f"resblock type {rtype} unrecognized.")

        # ---- encoder
        pyr_ch = channels
        add(conv3x3(channels, nf), "conv_in")
        hs_c = [nf]
        in_ch = nf
        for lvl in range(nres):
            for _ in range(nrb):
                out_ch = nf * ch_mult[lvl]
                add(Res(in_ch=in_ch, out_ch=out_ch), "res", "top")
                in_ch = out_ch
                if res_at[lvl] in attn_res:
                    add(Attn(channels=in_ch), "attn")
                hs_c.append(in_ch)
                plan.append(("push",))
            if lvl != nres - 1:
                if rtype == "ddpm":
                    add(Down(in_ch=in_ch), "resample_top")
                else:
                    add(Res(down=True, in_ch=in_ch), "res", "top")
                if prog_in == "input_skip":
                    add(layerspp.Combine(dim1=pyr_ch, dim2=in_ch, method=combine), "combine_in")
                    if combine == "cat":
                        in_ch *= 2
                elif prog_in == "residual":
                    add(pyr_down(in_ch=pyr_ch, out_ch=in_ch), "pyr_down")
                    pyr_ch = in_ch
                hs_c.append(in_ch)
                plan.append(("push",))

        # ---- bottleneck
        in_ch = hs_c[-1]
        plan.append(("h_from_top",))
        add(Res(in_ch=in_ch), "res", "h")
        add(Attn(channels=in_ch), "attn")
        add(Res(in_ch=in_ch), "res", "h")

        # ---- decoder
        pyr_ch = 0
        for lvl in reversed(range(nres)):
            for _ in range(nrb + 1):
                out_ch = nf * ch_mult[lvl]
                add(Res(in_ch=in_ch + hs_c.pop(), out_ch=out_ch), "res_cat")
                in_ch = out_ch
            if res_at[lvl] in attn_res:
                add(Attn(channels=in_ch), "attn")
            if prog != "none":
                gn = lambda c: nn.GroupNorm(num_groups=min(c // 4, 32), num_channels=c, eps=1e-6)
                if lvl == nres - 1:
                    gi = add(gn(in_ch))
                    if prog == "output_skip":
                        ci = add(conv3x3(in_ch, channels, init_scale=init_scale))
                        pyr_ch = channels
                    else:
                        ci = add(conv3x3(in_ch, in_ch, bias=True))
                        pyr_ch = in_ch
                    plan.append(("pyr_head", gi, ci))
                elif prog == "output_skip":
                    gi = add(gn(in_ch))
                    ci = add(conv3x3(in_ch, channels, bias=True, init_scale=init_scale))
                    pyr_ch = channels
                    plan.append(("pyr_out_skip", gi, ci))
                else:
                    add(pyr_up(in_ch=pyr_ch, out_ch=in_ch), "pyr_up")
                    pyr_ch = in_ch
            if lvl != 0:
                if rtype == "ddpm":
                    add(Up(in_ch=in_ch), "resample_h")
                else:
                    add(Res(in_ch=in_ch, up=True), "res", "h")
        assert not hs_c

        if prog != "output_skip":
            gi = add(nn.GroupNorm(num_groups=min(in_ch // 4, 32), num_channels=in_ch, eps=1e-6))
            ci = add(conv3x3(in_ch, channels, init_scale=init_scale))
            plan.append(("head", gi, ci))
        else:
            plan.append(("head_pyramid",))
        self.all_modules = nn.ModuleList(mods)
        self._plan = plan
        self._denses = None  # residual blocks' Dense_0, for layers.TembBank

    # ------------------------------------------------------------------
    def _time_embedding(self, time_cond):
        mods = self.all_modules
        if self.embedding_type == "fourier":
            used_sigmas = time_cond
            temb = mods[self._temb_idx](torch.log(used_sigmas))
        else:
            used_sigmas = None
            temb = layers.get_timestep_embedding(time_cond, self.nf)
        if self.conditional:
            temb = layers.dense(mods[self._dense_idx[0]], temb)
            temb = layers.dense(mods[self._dense_idx[1]], self.act(temb))
        else:
            temb = None
        return temb, used_sigmas

    def _gn_act_conv(self, h, gn, conv):
        """conv(act(GroupNorm(h))) -- the pyramid / output heads (reference ncsnpp.py:
        `self.act(modules[m_idx](h))` then conv3x3).  At inference the normalization is
        applied inside the conv's input load (statistics pass + conv, op.conv pre=)."""
        if layers.fused_inference_ok(self, h, self.act):
            y = layers.gn_silu_conv(h, gn, conv, conv_bias=conv.bias)
            if y is not None:
                return y
        return conv(layers.gn_act(h, gn, self.act))

    def forward(self, x, time_cond):
        mods = self.all_modules
        temb, used_sigmas = self._time_embedding(time_cond)
        if temb is not None and _TEMB_BANK and x.is_cuda and (
                layers._TEMB_BANK_AD or layers.fused_inference_ok(self, x, self.act)):
            if self._denses is None:
                self._denses = [m.Dense_0 for m in self.all_modules
                                if hasattr(m, "Dense_0") and isinstance(m.Dense_0, nn.Linear)]
            temb = layers.TembBank(temb, self.act, self._denses)
        if not self.config.data.centered:
            x = 2 * x - 1.
        pyramid = x if self.progressive_input != "none" else None
        hs: list = []
        h = x
        for step in self._plan:
            kind = step[0]
            if kind == "conv_in":
                h = mods[step[1]](x)
                hs.append(h)
            elif kind == "res":
                inp = hs[-1] if step[2] == "top" else h
                h = mods[step[1]](inp, temb)
            elif kind == "attn":
                h = mods[step[1]](h)
            elif kind == "push":
                hs.append(h)
            elif kind == "resample_top":
                h = mods[step[1]](hs[-1])
            elif kind == "resample_h":
                h = mods[step[1]](h)
            elif kind == "combine_in":
                pyramid = self.pyramid_downsample(pyramid)
                h = mods[step[1]](pyramid, h)
            elif kind == "pyr_down":
                pyramid = mods[step[1]](pyramid)
                pyramid = residual_rescale(pyramid, h, None, _SQRT2 if self.skip_rescale else 1.0)
                h = pyramid
            elif kind == "h_from_top":
                h = hs[-1]
            elif kind == "res_cat":
                blk = mods[step[1]]
                if hasattr(blk, "forward_pair") and _PAIR:
                    h = blk.forward_pair(h, hs.pop(), temb)
                else:
                    h = blk(layers.cat_channels(h, hs.pop()), temb)
            elif kind == "pyr_head":
                pyramid = self._gn_act_conv(h, mods[step[1]], mods[step[2]])
            elif kind == "pyr_out_skip":
                pyramid = self.pyramid_upsample(pyramid)
                ph = self._gn_act_conv(h, mods[step[1]], mods[step[2]])
                pyramid = pyramid + ph
            elif kind == "pyr_up":
                pyramid = mods[step[1]](pyramid)
                pyramid = residual_rescale(pyramid, h, None, _SQRT2 if self.skip_rescale else 1.0)
                h = pyramid
            elif kind == "head":
                h = self._gn_act_conv(h, mods[step[1]], mods[step[2]])
            elif kind == "head_pyramid":
                h = pyramid
            else:  # pragma: no cover
                raise RuntimeError(f"bad plan step {kind}")
        assert not hs
        if self.config.model.scale_by_sigma:
            if used_sigmas is None:
                used_sigmas = self.sigmas[time_cond.long()]
            h = h / used_sigmas.reshape((x.shape[0], *([1] * len(x.shape[1:]))))
        return h
