"""PINN flow / pressure networks (reference: models/flownet.py).

FlowNet: a shared 5-level feature pyramid for both frames, then coarse-to-fine
inference units (cost-volume matching on the HIP correlation kernel + sub-pixel
refinement), each warping frame-2 features with the current flow through the
HIP grid_sample (which carries the second derivative the PINN residual needs),
and a final bilinear upsample + residual conv head.  PressureNet: a residual
U-Net over |flow|^2 features.  Module nesting and parameter names follow the
reference exactly (so reference checkpoints load with strict=True, and a
seeded construction draws the same initial weights); the arithmetic differs only
where the HIP ops replace CuPy/CUDA extensions.

Call sites of the native ops: `project` -> op.grid_sample.grid_sample_2d
(reference flownet.py:21), `Matching` -> op.correlation.FunctionCorrelation
(reference flownet.py:117).
"""
from __future__ import annotations

import functools
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from op import channels, correlation, grid_sample
from op.fused_act import LeakyReLU, leaky_relu

from . import layers

_BASE_GRIDS: dict = {}
# FlowNet: the two frames' feature pyramids as one batch (A/B switch; tests flip it)
_PAIR_FRAMES = os.environ.get("BPK_PAIR_FRAMES", "1") == "1"


def _base_grid(shape, device):
    """Identity sampling grid [B, 2, H, W] in [-1, 1] (x then y), cached per shape and
    device (the reference caches a CPU copy and re-uploads it every call, flownet.py:7-14)."""
    key = (tuple(shape), str(device))
    g = _BASE_GRIDS.get(key)
    if g is None:
        B, _, H, W = shape
        gx = torch.linspace(-1.0, 1.0, W, device=device).view(1, 1, 1, W).expand(B, 1, H, W)
        gy = torch.linspace(-1.0, 1.0, H, device=device).view(1, 1, H, 1).expand(B, 1, H, W)
        g = torch.cat([gx, gy], 1)
        _BASE_GRIDS[key] = g
    return g


def project(f, u, dt):
    """Backward-warp f by the flow u over dt (reference flownet.py:8-25).

    The flow's channel 1 drives the x (width) coordinate and channel 0 the y
    coordinate, each normalised by (size - 1) / 2 of f's dims 2 and 3 respectively,
    exactly as the reference pairs them; border padding, align_corners=True.
    """
    grid = _base_grid(u.shape, u.device)
    # torch.cat([u[:, 1:2] / .., u[:, 0:1] / ..], 1) as one op in every derivative order
    step = channels.swap_scale(u, (f.size(2) - 1.0) / 2.0, (f.size(3) - 1.0) / 2.0)
    return grid_sample.grid_sample_2d(input=f, grid=(grid - step * dt).permute(0, 2, 3, 1),
                                      padding_mode="border", align_corners=True)


def _lrelu():
    # nn.LeakyReLU(0.1) of the reference, on the native kernel (op.fused_act.LeakyReLU)
    return LeakyReLU(negative_slope=0.1)


def _conv3(cin, cout, stride=1):
    # layers.Conv2d: nn.Conv2d parameters / state-dict keys, forward dispatched to the native
    # conv kernels where the shape qualifies (small-channel heads, Winograd), MIOpen otherwise
    return layers.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1)


def _chain(widths, last_act=False):
    """conv3x3 stack over consecutive widths with LeakyReLU(0.1) between convs."""
    mods = []
    for i, (cin, cout) in enumerate(zip(widths[:-1], widths[1:])):
        mods.append(_conv3(cin, cout))
        if last_act or i < len(widths) - 2:
            mods.append(_lrelu())
    return nn.Sequential(*mods)


def get_conv_feature_layer(in_channels, out_channels):
    """stride-2 conv + conv, LeakyReLU after each (reference flownet.py:27-33)."""
    return nn.Sequential(_conv3(in_channels, out_channels, 2), _lrelu(),
                         _conv3(out_channels, out_channels), _lrelu())


def get_conv_decode_layer(in_channels, out_channels):
    return _chain([in_channels, out_channels], last_act=True)


def get_conv_field_layer(in_channels, out_channels):
    """in -> 128 -> 64 -> 32 -> out (reference flownet.py:42-50)."""
    return _chain([in_channels, 128, 64, 32, out_channels])


def get_conv_up_layer(out_channels):
    """(2 + out) -> 64 -> 32 -> out (reference flownet.py:52-58)."""
    return _chain([2 + out_channels, 64, 32, out_channels])


class FeatureExtractor(nn.Module):
    """Pyramid of stride-2 conv pairs; before each level the input gets the spatial
    embedding (average-pooled per level) and a timestep embedding of its own width
    (reference flownet.py:60-90)."""

    def __init__(self, config):
        super().__init__()
        widths = [config.data.num_channels] + list(config.model.feature_nums)
        self.fln = len(widths) - 1
        self.spatial_emb = functools.partial(layers.get_spatial_embedding,
                                             omega=config.model.spatial_embed_omega,
                                             s=config.model.spatial_embed_s_flow)
        self.semb_down = nn.AvgPool2d(kernel_size=2, stride=2, padding=0)
        self.feature_extractors = nn.ModuleList(
            get_conv_feature_layer(a, b) for a, b in zip(widths[:-1], widths[1:]))

    def embeddings(self, x, y, t, channels_in):
        """The (spatial, timestep) embedding added before each level: the same tensors for
        both frames, so FlowNet computes them once (the reference builds them per frame:
        identical values, and every derivative pass of the PINN residual then runs through
        one copy of the sin / sqrt / pool chain instead of two)."""
        dims = [channels_in] + [level[-2].out_channels for level in self.feature_extractors][:-1]
        tembs = layers.get_timestep_embeddings(t, dims)  # every level's in one chain
        out, semb = [], self.spatial_emb(x, y)
        for temb in tembs:
            out.append((semb, temb[:, :, None, None]))
            semb = self.semb_down(semb)
        return out

    def forward(self, f, x, y, t, emb=None):
        pyramid = []
        if emb is None:
            emb = self.embeddings(x, y, t, f.shape[1])
        for level, (semb, temb) in zip(self.feature_extractors, emb):
            f = level(f + semb + temb)
            pyramid.append(f)
        return pyramid

    def forward_frames(self, frames, emb):
        """The pyramids of k frames [k, B, C, H, W] (stacked along the batch) in one pass per
        level: the same weights and embeddings for every frame, so each conv / activation runs
        once at batch k*B instead of k times at B -- in the forward and in every derivative
        pass of the PINN residual.  Per-sample arithmetic and the reference's add order
        ((f + semb) + temb, broadcast over the frames); returns k pyramids."""
        k, B = frames.shape[0], frames.shape[1]
        f = frames.reshape((k * B,) + tuple(frames.shape[2:]))
        levels = []
        for level, (semb, temb) in zip(self.feature_extractors, emb):
            h = f.view((k, B) + tuple(f.shape[1:])) + semb[None] + temb[None]
            f = level(h.view((k * B,) + tuple(f.shape[1:])))
            levels.append(channels.split(f, (B,) * k, 0))
        return [list(p) for p in zip(*levels)]


class Matching(nn.Module):
    """Cost-volume flow estimate at one level (reference flownet.py:93-121)."""

    def __init__(self, config, level):
        super().__init__()
        self.dt = config.data.dt * 0.5 ** level
        self.flow_upsample = layers.ConvTranspose2d(2, 2, kernel_size=4, stride=2, padding=1,
                                                    bias=False, groups=2)
        self.corr_conv = get_conv_field_layer(49, 2)

    def forward(self, feature1, feature2, flow=None):
        if flow is None:
            base = 0.0
        else:
            base = self.flow_upsample(flow)
            feature2 = project(feature2, base, -self.dt)
        cost = leaky_relu(correlation.FunctionCorrelation(feature1, feature2, stride=1))
        return base + self.corr_conv(cost)


class SubpixelRefinement(nn.Module):
    """Residual flow correction from [f1, warped f2, flow] (reference flownet.py:123-138)."""

    def __init__(self, config, level):
        super().__init__()
        self.dt = config.data.dt * 0.5 ** (level + 1)
        self.flow_conv = get_conv_field_layer(config.model.feature_nums[level] * 2 + 2, 2)

    def forward(self, feature1, feature2, flow):
        warped = project(feature2, flow, -self.dt)
        return flow + self.flow_conv(channels.cat([feature1, warped, flow], dim=1))


class InferenceUnit(nn.Module):
    def __init__(self, config, level):
        super().__init__()
        self.level = level
        self.match = Matching(config, level)
        self.refinement = SubpixelRefinement(config, level)

    def forward(self, feature1, feature2, flow=None, p_prev=None):
        return self.refinement(feature1, feature2, self.match(feature1, feature2, flow))


class Upsample(nn.Module):
    """Bilinear upsample of the finest flow + conv residual (reference flownet.py:151-163)."""

    def __init__(self):
        super().__init__()
        self.up = get_conv_up_layer(2)

    def forward(self, f1, f2, x, size):
        x = F.interpolate(input=x, size=size, mode="bilinear", align_corners=False)
        return x + self.up(channels.cat([f1, f2, x], dim=1))


class FlowNet(nn.Module):
    """forward(f1, f2, x, y, t) -> cascaded flows, coarsest first, full-size last
    (reference flownet.py:166-193)."""

    def __init__(self, config):
        super().__init__()
        self.size = (config.data.image_size, config.data.image_size)
        self.feature_extractor = FeatureExtractor(config)
        n = len(config.model.feature_nums)
        self.inference_units = nn.ModuleList(InferenceUnit(config, lv)
                                             for lv in reversed(range(n)))
        self.upsample = Upsample()

    def forward(self, f1, f2, x, y, t, size=None):
        emb = self.feature_extractor.embeddings(x, y, t, f1.shape[1])
        if _PAIR_FRAMES and f1.is_cuda:
            # both frames through the shared extractor as one batch (forward_frames)
            p1, p2 = self.feature_extractor.forward_frames(torch.stack([f1, f2]), emb)
        else:
            p1 = self.feature_extractor(f1, x, y, t, emb)
            p2 = self.feature_extractor(f2, x, y, t, emb)
        flows, flow = [], None
        for unit in self.inference_units:
            flow = unit(p1[unit.level], p2[unit.level], flow)
            flows.append(flow)
        flows.append(self.upsample(f1, f2, flow, self.size if size is None else size))
        return flows

    def multiscale_data_mse(self, veloc_pred, target, error_fn=torch.nn.MSELoss()):
        """Weighted MSE of each cascade level against a bilinearly shrunk target; level i
        (from the finest) is scaled by 2^-i (reference flownet.py:195-216)."""
        weights = [12.7, 5.5, 4.35, 3.9, 3.4, 1.1][:len(veloc_pred)]
        h, w = veloc_pred[-1].shape[-2:]
        total = 0
        for i, wt in enumerate(weights):
            scale = 1.0 / (2 ** i)
            total = total + wt * error_fn(veloc_pred[-1 - i] * scale, target[:, :2] * scale)
            h, w = h // 2, w // 2
            target = F.interpolate(target, (h, w), mode="bilinear", align_corners=False)
        return total


def get_double_res(in_channels, out_channels, num_groups=16):
    """Two ResidualBlocks: in -> 2*in -> out (reference flownet.py:219-224)."""
    return nn.Sequential(layers.ResidualBlock(in_channels, in_channels * 2),
                         layers.ResidualBlock(in_channels * 2, out_channels))


def get_down_layer(in_channels, out_channels):
    return nn.Sequential(nn.MaxPool2d(2), get_double_res(in_channels, out_channels))


def get_up_layer(in_channels, out_channels):
    return nn.Sequential(layers.ConvTranspose2d(in_channels, out_channels, kernel_size=2, stride=2))


class PressureNet(nn.Module):
    """forward(cascaded_flow, x, y, t) -> pressure [B, 1, H, W] (reference flownet.py:237-318)."""

    def __init__(self, config):
        super().__init__()
        self.channels = ch = list(config.model.feature_nums)
        self.flow_feature_nums = ff = 32
        self.flow_feature = get_double_res(3, ff)
        self.spatial_emb = functools.partial(layers.get_spatial_embedding,
                                             omega=config.model.spatial_embed_omega,
                                             s=config.model.spatial_embed_s_pres)
        self.semb_down = nn.AvgPool2d(kernel_size=2, stride=2, padding=0)
        self.first = get_double_res(ff, ch[0])
        self.down = nn.ModuleList(get_down_layer(a, b) for a, b in zip(ch[:-1], ch[1:]))
        ups, up_convs = [], []
        for cin, cout in zip(ch[:0:-1], ch[-2::-1]):
            ups.append(get_up_layer(cin, cout))
            up_convs.append(get_double_res(cout * 2 + ff, cout, 4))
        self.up = nn.ModuleList(ups)
        self.up_conv = nn.ModuleList(up_convs)
        half = ch[0] // 2
        self.end = nn.Sequential(get_double_res(ch[0], half),
                                 layers.Conv2d(half, half, kernel_size=1),
                                 get_double_res(half, 1), layers.Conv2d(1, 1, kernel_size=1))

    def get_norm_feature(self, flow):
        """features of [u, v, -(u^2 + v^2)] (reference flownet.py:280-283)."""
        return self.flow_feature(channels.cat([flow, -(flow ** 2).sum(dim=1, keepdim=True)], dim=1))

    def get_semb_list(self, x, y):
        out = [self.spatial_emb(x, y)]
        for _ in range(len(self.channels) - 2):
            out.append(self.semb_down(out[-1]))
        return out

    def forward(self, cascaded_flow, x, y, t):
        temb = layers.get_timestep_embedding(t, self.flow_feature_nums)[:, :, None, None]
        semb = self.get_semb_list(x, y)
        h = self.first(self.get_norm_feature(cascaded_flow[-1].detach().clone()) + temb + semb[0])
        skips = [h]
        for down in self.down:
            h = down(h)
            skips.append(h)
        skips.pop()
        for i, (up, up_conv) in enumerate(zip(self.up, self.up_conv)):
            ffeat = self.get_norm_feature(cascaded_flow[i + 2].detach().clone()) + temb + semb[-1 - i]
            h = up_conv(channels.cat([skips[-1 - i], up(h), ffeat], dim=1))
        return self.end(h)

    def data_mse(self, pressure, target, error_fn=torch.nn.MSELoss()):
        return error_fn(pressure, target[:, 2:3])
