"""Navier-Stokes / PINN rollouts (reference pinn_kalman/simulator.py:6-63).

`step(model, begin, t_range, stride)` advances B = 256 replicas of the 192x192 fields
of one snapshot with the ns_step stencil (dt = 0.0025, dx = 1/200), returning the
per-step density, velocity and pressure; `simulate(model, begin, ...)` rolls the PINN
forward (FlowNet flow -> `PINN.step` warp).  `begin` is the dataset array
[T, 6, H, W] (channels x, y, f, u, v, p), cropped as the reference does ([8:200, 4:-4]).

MI355X design: one simulator step is the fused `ns_step.full_step` (two launches,
bit-identical to the reference's three ops), the replicas stay resident in HBM, and the
reference's per-step `print(f)` (a device sync + host transfer of 9.4 M values) is dropped.
"""
from __future__ import annotations

import numpy as np
import torch

from op import ns_step

dt = 0.0005 * 5
dx = 1 / 200


def _prep(data, device):
    return torch.from_numpy(np.ascontiguousarray(data[:, 8:200, 4:-4])).to(device).unsqueeze(0)


def simulate(model, begin, t_range=(0, 100), stride=1):
    dev = model.mask_u.device
    t0, _ = t_range
    f1 = _prep(begin[0 + t0, 2:3], dev)
    f2 = _prep(begin[1 + t0, 2:3], dev)
    x = _prep(begin[0 + t0, 0:1], dev)
    y = _prep(begin[0 + t0, 1:2], dev)
    result, vel = [], []
    for t in torch.arange(*t_range, stride):
        t = t.unsqueeze(0).to(dev)
        flow, _ = model(f1, f2, x, y, t, size=(192, 192))
        f = model.step(f2, flow[-1])
        result.append(f)
        vel.append(flow[-1])
        f1, f2 = f2, f
    return result, vel


def step(model, begin, t_range=(0, 100), stride=1, replicas=256, device=None, ctx=None,
         compat=True):
    """ns_step rollout of `replicas` copies of snapshot t_range[0]; velocity channels are
    swapped into (v, u) order as the reference does (simulator.py:52-53).

    ctx (dist.DistContext): batch-sharded over the ranks, no collective -- rank r advances
    replicas [r * R, (r + 1) * R) with R = replicas / world and returns those.
    compat=False: replicas are independent and the shards equal the single-process rollout
    bit for bit.  compat=True (the reference's behaviour): update_velocity's unbind quirk
    (op/ns_step.cpp:70) makes sample b advect velocity planes b and b + 1, i.e. samples
    b / 2 and (b + 1) / 2, so the replicas diverge after the first step and a shard equals
    the reference's own rollout of R replicas -- reproducing the single-process batch would
    need every rank's velocities each step."""
    dev = device if device is not None else model.mask_u.device
    t0, _ = t_range
    if ctx is not None and ctx.enabled:
        if replicas % ctx.world_size:
            raise ValueError(f"replicas {replicas} do not split over {ctx.world_size} ranks")
        replicas //= ctx.world_size
    f = _prep(begin[0 + t0, 2:3], dev).repeat(replicas, 1, 1, 1)
    v = _prep(begin[0 + t0, 3:5], dev)
    v = torch.cat([v[:, 1:2], v[:, 0:1]], 1).repeat(replicas, 1, 1, 1)
    p = _prep(begin[0 + t0, 5:6], dev).repeat(replicas, 1, 1, 1)
    result, vel, pres = [], [], []
    for _ in torch.arange(*t_range, stride):
        f, v, p = ns_step.full_step(f, v, p, dt, dx, compat=compat)
        result.append(f)
        vel.append(v)
        pres.append(p)
    return result, vel, pres
