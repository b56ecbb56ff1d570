"""ORACLE (test infrastructure only) -- the deterministic PINN restated on torch-CPU.

FlowNet + PressureNet (reference models/flownet.py:8-321), the Navier-Stokes residual
(pinn_kalman/pinn.py:72-111) and the PINN train step (losses.py:332-386) as plain aten CPU
ops over a parameter dict (the product PINN's state dict, same keys as the reference).
The two CUDA-only pieces of the reference are the oracle restatements:
  * correlation (CuPy, op/correlation.py): stride-1 cost volume vectorised in torch,
    first-order only exactly as the reference (its backward is not differentiable);
    checked against oracle/correlation_ref.py in tests/test_pinn_ref.py;
  * grid_sample (op/grid_sample.py:15-131): aten forward / backward, double backward from
    oracle/grid_sample_ref.grad2.
Pinned against the reference-generated fixtures tests/golden/pinn_fwd.npz (16^2) and
cfg_pinn64.npz (configs[3] at 64^2) in tests/test_pinn_ref.py.  Used by bench.py as the
PINN row's CPU baseline; never by the product path.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import grid_sample_ref


# ------------------------------------------------------------------ native-op stand-ins

class _GridSampleBwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gout, inp, grid):
        ctx.save_for_backward(gout, inp, grid)
        return grid_sample_ref.bwd(gout, inp, grid, padding_mode=1, align_corners=True)

    @staticmethod
    def backward(ctx, g2_inp, g2_grid):
        gout, inp, grid = ctx.saved_tensors
        if g2_inp is None:
            g2_inp = torch.zeros_like(inp)
        if g2_grid is None:
            g2_grid = torch.zeros_like(grid)
        ggo, gi, gg = grid_sample_ref.grad2(g2_inp, g2_grid, gout, inp, grid, 1, True)
        return ggo, gi, gg


class _GridSample(torch.autograd.Function):
    """border padding, align_corners=True (the only mode `project` uses, flownet.py:21-25)"""

    @staticmethod
    def forward(ctx, inp, grid):
        ctx.save_for_backward(inp, grid)
        return grid_sample_ref.fwd(inp, grid, padding_mode=1, align_corners=True)

    @staticmethod
    def backward(ctx, gout):
        inp, grid = ctx.saved_tensors
        return _GridSampleBwd.apply(gout.contiguous(), inp, grid)


def _corr_fwd(a, b):
    """out[:, (dy+3)*7 + dx+3] = mean_c a[c, y, x] * b[c, y+dy, x+dx], zero outside
    (CuPy kernel_Correlation_updateOutput, op/correlation.py:34-102, stride 1)."""
    B, C, H, W = a.shape
    bp = F.pad(b, (3, 3, 3, 3))
    out = a.new_empty((B, 49, H, W))
    for tc in range(49):
        dy, dx = tc // 7, tc % 7
        out[:, tc] = (a * bp[:, :, dy:dy + H, dx:dx + W]).sum(1) / C
    return out


class _Correlation(torch.autograd.Function):
    """First-order only, as the reference (its CuPy backward is not differentiable)."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return _corr_fwd(a, b)

    @staticmethod
    def backward(ctx, g):
        # computed on detached values: constant to any further derivative (second-order
        # terms through the cost volume vanish, as with the reference's CuPy backward)
        a, b = (v.detach() for v in ctx.saved_tensors)
        g = g.detach()
        B, C, H, W = a.shape
        bp = F.pad(b, (3, 3, 3, 3))
        ga = torch.zeros_like(a)
        gbp = torch.zeros_like(bp)
        for tc in range(49):
            dy, dx = tc // 7, tc % 7
            gt = g[:, tc:tc + 1] / C
            ga += gt * bp[:, :, dy:dy + H, dx:dx + W]
            gbp[:, :, dy:dy + H, dx:dx + W] += gt * a
        return ga, gbp[:, :, 3:3 + H, 3:3 + W]


def correlation(a, b):
    return _Correlation.apply(a, b)


# ------------------------------------------------------------------ building blocks

def timestep_embedding(t, dim, max_positions=10000):
    """reference models/layers.py:500-514"""
    half = dim // 2
    e = math.log(max_positions) / (half - 1)
    e = torch.exp(torch.arange(half, dtype=torch.float32) * -e)
    e = t.float()[:, None] * e[None, :]
    e = torch.cat([torch.sin(e), torch.cos(e)], dim=1)
    if dim % 2 == 1:
        e = F.pad(e, (0, 1))
    return e


def spatial_embedding(x, y, omega, s):
    """reference models/layers.py:517-521"""
    e1 = torch.sin(omega * torch.sqrt(x ** 2 + y ** 2))
    e2 = torch.sin(omega * torch.sqrt((x.max() - x) ** 2 + (y.max() - y) ** 2))
    return (e1 + e2) / s


def project(f, u, dt):
    """reference flownet.py:8-25"""
    B, _, H, W = u.shape
    gh = torch.linspace(-1.0, 1.0, W).view(1, 1, 1, W).expand(B, -1, H, -1)
    gv = torch.linspace(-1.0, 1.0, H).view(1, 1, H, 1).expand(B, -1, -1, W)
    grid = torch.cat([gh, gv], 1)
    u = torch.cat([u[:, 1:2] / ((f.size(2) - 1.0) / 2.0), u[:, 0:1] / ((f.size(3) - 1.0) / 2.0)], 1)
    return _GridSample.apply(f, (grid - u * dt).permute(0, 2, 3, 1))


def _conv(P, pre, x, stride=1, padding=1):
    return F.conv2d(x, P[pre + "weight"], P.get(pre + "bias"), stride=stride, padding=padding)


def _lrelu(x):
    return F.leaky_relu(x, 0.1)


def _chain(P, pre, x, n):
    """conv(0) lrelu conv(2) lrelu ... conv(2n-2) (get_conv_field_layer / up_layer,
    flownet.py:41-57)"""
    for i in range(n):
        x = _conv(P, f"{pre}{2 * i}.", x)
        if i < n - 1:
            x = _lrelu(x)
    return x


# ------------------------------------------------------------------ FlowNet

def flownet(P, cfg, f1, f2, x, y, t, size=None):
    """reference flownet.py:60-193 -> cascaded flows, coarsest first, full size last"""
    m = cfg.model
    n = len(m.feature_nums)

    def features(f):
        out = []
        semb = spatial_embedding(x, y, m.spatial_embed_omega, m.spatial_embed_s_flow)
        for i in range(n):
            temb = timestep_embedding(t, f.shape[1])[:, :, None, None]
            pre = f"flownet.feature_extractor.feature_extractors.{i}."
            f = _lrelu(_conv(P, pre + "0.", f + semb + temb, stride=2))
            f = _lrelu(_conv(P, pre + "2.", f))
            out.append(f)
            semb = F.avg_pool2d(semb, 2, 2)
        return out

    p1, p2 = features(f1), features(f2)
    flows, flow = [], None
    for j, level in enumerate(reversed(range(n))):
        pre = f"flownet.inference_units.{j}."
        a, b = p1[level], p2[level]
        dt = cfg.data.dt * 0.5 ** level
        if flow is not None:
            base = F.conv_transpose2d(flow, P[pre + "match.flow_upsample.weight"], stride=2,
                                      padding=1, groups=2)
            b_w = project(b, base, -dt)
        else:
            base, b_w = 0.0, b
        flow = base + _chain(P, pre + "match.corr_conv.", _lrelu_corr(correlation(a, b_w)), 4)
        warped = project(b, flow, -cfg.data.dt * 0.5 ** (level + 1))
        flow = flow + _chain(P, pre + "refinement.flow_conv.", torch.cat([a, warped, flow], 1), 4)
        flows.append(flow)
    size = (cfg.data.image_size, cfg.data.image_size) if size is None else size
    up = F.interpolate(flow, size=size, mode="bilinear", align_corners=False)
    flows.append(up + _chain(P, "flownet.upsample.up.", torch.cat([f1, f2, up], 1), 3))
    return flows


def _lrelu_corr(c):
    return F.leaky_relu(c)  # default slope 0.01 (flownet.py:119)


# ------------------------------------------------------------------ PressureNet

def _resblock(P, pre, x):
    """ResidualBlock, resample=None (reference layers.py:438-492): IN -> ELU -> conv3x3 ->
    IN -> ELU -> conv3x3, + identity or 1x1 shortcut"""
    h = _conv(P, pre + "conv1.", F.elu(F.instance_norm(x, eps=1e-5)))
    h = _conv(P, pre + "conv2.", F.elu(F.instance_norm(h, eps=1e-5)))
    skip = _conv(P, pre + "shortcut.", x, padding=0) if pre + "shortcut.weight" in P else x
    return skip + h


def _double(P, pre, x):
    return _resblock(P, pre + "1.", _resblock(P, pre + "0.", x))


def pressurenet(P, cfg, flows, x, y, t):
    """reference flownet.py:237-318"""
    m = cfg.model
    ch = list(m.feature_nums)
    temb = timestep_embedding(t, 32)[:, :, None, None]
    semb = [spatial_embedding(x, y, m.spatial_embed_omega, m.spatial_embed_s_pres)]
    for _ in range(len(ch) - 2):
        semb.append(F.avg_pool2d(semb[-1], 2, 2))

    def norm_feature(fl):
        fl = fl.detach().clone()
        return _double(P, "pressurenet.flow_feature.",
                       torch.cat([fl, -(fl ** 2).sum(dim=1).unsqueeze(1)], 1))

    h = _double(P, "pressurenet.first.", norm_feature(flows[-1]) + temb + semb[0])
    feats = [h]
    for i in range(len(ch) - 1):
        h = _double(P, f"pressurenet.down.{i}.1.", F.max_pool2d(h, 2))
        feats.append(h)
    feats.pop()
    for i in range(len(feats)):
        ff = norm_feature(flows[i + 2]) + temb + semb[-1 - i]
        pre = f"pressurenet.up.{i}.0."
        u = F.conv_transpose2d(h, P[pre + "weight"], P[pre + "bias"], stride=2)
        h = _double(P, f"pressurenet.up_conv.{i}.", torch.cat([feats[-1 - i], u, ff], 1))
    h = _double(P, "pressurenet.end.0.", h)
    h = _conv(P, "pressurenet.end.1.", h, padding=0)
    h = _double(P, "pressurenet.end.2.", h)
    return _conv(P, "pressurenet.end.3.", h, padding=0)


def forward(P, cfg, f1, f2, x, y, t):
    flows = flownet(P, cfg, f1, f2, x, y, t)
    return flows, pressurenet(P, cfg, flows, x, y, t)


# ------------------------------------------------------------------ residual and step

def equation_mse(x, y, t, flow, pres, Re):
    """reference pinn.py:72-111 (u, v by 'differentiable slicing' = channel selection)"""
    u, v, p = flow[:, 0:1] * 1.0, flow[:, 1:2] * 1.0, pres
    g = torch.autograd.grad
    u_x, u_y, u_t = g(u.sum(), (x, y, t), create_graph=True, retain_graph=True)
    v_x, v_y, v_t = g(v.sum(), (x, y, t), create_graph=True, retain_graph=True)
    p_x, p_y = g(p.sum(), (x, y), create_graph=True, retain_graph=True)
    u_xx = g(u_x.sum(), x, retain_graph=True)[0]
    u_yy = g(u_y.sum(), y, retain_graph=True)[0]
    v_xx = g(v_x.sum(), x, retain_graph=True)[0]
    v_yy = g(v_y.sum(), y, retain_graph=True)[0]
    u_t = u_t[:, None, None, None]
    v_t = v_t[:, None, None, None]
    nu = 1.0 / Re
    res_x = u_t + (u * u_x + v * u_y) + p_x - nu * (u_xx + u_yy)
    res_y = v_t + (u * v_x + v * v_y) + p_y - nu * (v_xx + v_yy)
    res_m = u_x + v_y
    return (res_x ** 2).mean() + (res_y ** 2).mean() + (res_m ** 2).mean()


def multiscale_data_mse(flows, target):
    """reference flownet.py:195-216"""
    h, w = flows[-1].shape[-2:]
    total = 0
    for i, wt in enumerate([12.7, 5.5, 4.35, 3.9, 3.4, 1.1][:len(flows)]):
        s = 1.0 / (2 ** i)
        total = total + wt * F.mse_loss(flows[-1 - i] * s, target[:, :2] * s)
        h, w = h // 2, w // 2
        target = F.interpolate(target, (h, w), mode="bilinear", align_corners=False)
    return total


def pinn_loss(P, cfg, batch, mask, noise):
    """reference losses.py:334-346: observed frames = mask * f + sqrt(var) * noise"""
    f1, f2, x, y, t, target = batch
    sd = cfg.inverse.variance ** 0.5
    f1 = mask * f1 + noise[0] * sd
    f2 = mask * f2 + noise[1] * sd
    flows, pres = forward(P, cfg, f1, f2, x, y, t)
    data = multiscale_data_mse(flows, target) + F.mse_loss(pres, target[:, 2:3])
    pinn = equation_mse(x, y, t, flows[-1], pres, 10000000.0) * cfg.training.pinn_loss_weight
    return pinn + data, pinn, data


def init_params(state_dict):
    """float32 CPU leaf tensors requiring grad, keyed like the reference state dict"""
    return {k: v.detach().to("cpu", torch.float32).clone().requires_grad_(v.is_floating_point())
            for k, v in state_dict.items()}
