"""ORACLE (test infrastructure only) -- InstanceNorm2d(affine=False) + ELU(alpha=1):
forward, backward and the analytic double backward restated in numpy (float64).

What it restates: PressureNet's ResidualBlock `conv(act(normalize(x)))` (reference
models/layers.py:438-491, InstanceNorm2d + nn.ELU) as aten differentiates it -- the
batch-norm statistics / backward and elu_backward (z <= 0 branch at z = 0).  The double
backward is the closed form the HIP kernel evaluates (csrc/instance_norm.hip header);
tests/test_oracle.py pins it against torch's own composite double backward on the CPU.
"""
from __future__ import annotations

import numpy as np


def _stats(x, eps):
    P = x.shape[0] * x.shape[1]
    xf = x.reshape(P, -1).astype(np.float64)
    mu = xf.mean(1, keepdims=True)
    r = 1.0 / np.sqrt(((xf - mu) ** 2).mean(1, keepdims=True) + eps)
    return xf, mu, r


def _d1(z, act):
    return np.where(z <= 0, np.exp(z), 1.0) if act else np.ones_like(z)


def _d2(z, act):
    return np.where(z <= 0, np.exp(z), 0.0) if act else np.zeros_like(z)


def forward(x, eps=1e-5, act=1):
    xf, mu, r = _stats(x, eps)
    z = (xf - mu) * r
    y = np.where(z <= 0, np.expm1(z), z) if act else z
    return y.reshape(x.shape)


def backward(dy, x, eps=1e-5, act=1):
    xf, mu, r = _stats(x, eps)
    z = (xf - mu) * r
    g = dy.reshape(z.shape) * _d1(z, act)
    dx = r * (g - g.mean(1, keepdims=True) - z * (g * z).mean(1, keepdims=True))
    return dx.reshape(x.shape)


def double_backward(v, dy, x, eps=1e-5, act=1):
    """(dL/d dy, dL/dx) for L = <v, backward(dy, x)>."""
    xf, mu, r = _stats(x, eps)
    z = (xf - mu) * r
    d1 = _d1(z, act)
    dyf = dy.reshape(z.shape)
    vf = v.reshape(z.shape)
    g = dyf * d1
    m = lambda a: a.mean(1, keepdims=True)
    mv, mvz, mg, mgz, mgv = m(vf), m(vf * z), m(g), m(g * z), m(g * vf)
    w = r * (vf - mv - z * mvz)
    gdy = w * d1
    q = dyf * _d2(z, act) * w - r * (g * mvz + vf * mgz)
    S = mgv - mg * mv - mgz * mvz
    gx = r * (q - m(q) - z * m(q * z)) - r * r * z * S
    return gdy.reshape(x.shape), gx.reshape(x.shape)
