"""Device-resident explicit Runge-Kutta solver with scipy's step-size control.

The reference integrates its probability-flow / DPS ODEs with
`scipy.integrate.solve_ivp(fun, (t1, eps), x0, rtol=1e-3, atol=1e-3, method='RK45')`
on a flattened float64 host copy of the state (inverse/conditional_sampling.py:10-19),
so every function evaluation copies the whole batch device->host->device.  Here the
state, the stage matrix K and all stage combinations stay in HBM (float64, as scipy
keeps them); the only host traffic per step is one scalar (the error norm) that the
step-size controller needs.  The controller reproduces scipy 1.15's RungeKutta
(`scipy/integrate/_ivp/rk.py` `_step_impl`, `rk_step`; `common.select_initial_step`;
`solve_ivp` loop), the version in this image (the reference pins scipy~=1.13.1, whose
RK45 controller is the same algorithm), so the accepted time grid and nfev match
scipy's on the same function (tests/test_dps_host.py).

`reduce_sumsq(t)` hooks the two global reductions (RMS norms) so a batch-sharded run
(one shard of the state per rank) takes rank-identical step decisions: pass a function
that all-reduces the local sum of squares.
"""
from __future__ import annotations

import math

import numpy as np
import torch

SAFETY = 0.9
MIN_FACTOR = 0.2
MAX_FACTOR = 10.0

# Dormand-Prince 5(4) (scipy RK45) and Bogacki-Shampine 3(2) (scipy RK23) tableaus
_RK45 = dict(
    order=5, err_order=4,
    C=[0.0, 1 / 5, 3 / 10, 4 / 5, 8 / 9, 1.0],
    A=[[],
       [1 / 5],
       [3 / 40, 9 / 40],
       [44 / 45, -56 / 15, 32 / 9],
       [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
       [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656]],
    B=[35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84],
    E=[-71 / 57600, 0.0, 71 / 16695, -71 / 1920, 17253 / 339200, -22 / 525, 1 / 40],
)
_RK23 = dict(
    order=3, err_order=2,
    C=[0.0, 1 / 2, 3 / 4],
    A=[[], [1 / 2], [0.0, 3 / 4]],
    B=[2 / 9, 1 / 3, 4 / 9],
    E=[5 / 72, -1 / 12, -1 / 9, 1 / 8],
)
TABLEAUS = {"RK45": _RK45, "RK23": _RK23}


class Solution:
    def __init__(self, t, y, nfev, status, message, n_steps):
        self.t, self.y, self.nfev = t, y, nfev
        self.status, self.message, self.n_steps = status, message, n_steps
        self.success = status >= 0


def _rms(x, n_global, reduce_sumsq):
    s = torch.sum(x * x)
    if reduce_sumsq is not None:
        s = reduce_sumsq(s)
    return math.sqrt(float(s) / n_global)


def solve_ivp_rk(fun, t_span, y0, method="RK45", rtol=1e-3, atol=1e-3, reduce_sumsq=None,
                 n_global=None, max_steps=None):
    """Integrate dy/dt = fun(t, y) from t_span[0] to t_span[1].

    fun(t: float, y: float64 tensor) -> tensor (any float dtype, same shape; cast to
    float64 like scipy's wrapper).  y0: tensor, stays on its device.  Returns a
    Solution whose .y is the final state (float64 tensor) -- the reference only ever
    reads `solution.y[:, -1]`.  `max_steps` bounds the number of accepted steps (for
    benchmarks); the solution then carries status 2 ("step budget reached").
    """
    tab = TABLEAUS[method]
    t0, t_bound = float(t_span[0]), float(t_span[1])
    direction = float(np.sign(t_bound - t0)) if t_bound != t0 else 1.0
    y = y0.to(torch.float64).reshape(-1).clone()
    n = y.numel() if n_global is None else n_global
    A, B, C, E = tab["A"], tab["B"], tab["C"], tab["E"]
    n_stages = len(C)
    err_exp = -1.0 / (tab["err_order"] + 1)
    nfev = [0]

    def f(t, yy):
        nfev[0] += 1
        return fun(t, yy).to(torch.float64).reshape(-1)

    t = t0
    fy = f(t, y)
    # select_initial_step (scipy common.py)
    interval = abs(t_bound - t0)
    if interval == 0.0:
        h_abs = 0.0
    else:
        scale = atol + torch.abs(y) * rtol
        d0 = _rms(y / scale, n, reduce_sumsq)
        d1 = _rms(fy / scale, n, reduce_sumsq)
        h0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
        h0 = min(h0, interval)
        y1 = y + h0 * direction * fy
        f1 = f(t0 + h0 * direction, y1)
        d2 = _rms((f1 - fy) / scale, n, reduce_sumsq) / h0
        if d1 <= 1e-15 and d2 <= 1e-15:
            h1 = max(1e-6, h0 * 1e-3)
        else:
            h1 = (0.01 / max(d1, d2)) ** (1 / (tab["err_order"] + 1))
        h_abs = min(100 * h0, h1, interval, math.inf)

    K = torch.empty((n_stages + 1, y.numel()), dtype=torch.float64, device=y.device)
    status, message, steps = None, "", 0
    if t == t_bound:
        status, message = 0, "The solver successfully reached the end of the integration interval."
    while status is None:
        min_step = 10 * abs(np.nextafter(t, direction * np.inf) - t)
        h_abs = min(max(h_abs, min_step), math.inf)
        accepted, rejected = False, False
        while not accepted:
            if h_abs < min_step:
                status, message = -1, "Required step size is less than spacing between numbers."
                break
            h = h_abs * direction
            t_new = t + h
            if direction * (t_new - t_bound) > 0:
                t_new = t_bound
            h = t_new - t
            h_abs = abs(h)
            # rk_step
            K[0] = fy
            for s in range(1, n_stages):
                dy = torch.zeros_like(y)
                for j, a in enumerate(A[s]):
                    if a != 0.0:
                        dy.add_(K[j], alpha=a)
                K[s] = f(t + C[s] * h, y + dy * h)
            acc = torch.zeros_like(y)
            for j, b in enumerate(B):
                if b != 0.0:
                    acc.add_(K[j], alpha=b)
            y_new = y + h * acc
            f_new = f(t + h, y_new)
            K[-1] = f_new
            scale = atol + torch.maximum(torch.abs(y), torch.abs(y_new)) * rtol
            err = torch.zeros_like(y)
            for j, e in enumerate(E):
                if e != 0.0:
                    err.add_(K[j], alpha=e)
            err_norm = _rms(err * h / scale, n, reduce_sumsq)
            if err_norm < 1:
                factor = MAX_FACTOR if err_norm == 0 else min(MAX_FACTOR,
                                                              SAFETY * err_norm ** err_exp)
                if rejected:
                    factor = min(1, factor)
                h_abs *= factor
                accepted = True
            else:
                h_abs *= max(MIN_FACTOR, SAFETY * err_norm ** err_exp)
                rejected = True
        if status is not None:
            break
        t, y, fy = t_new, y_new, f_new
        steps += 1
        if direction * (t - t_bound) >= 0:
            status, message = 0, "The solver successfully reached the end of the integration interval."
        elif max_steps is not None and steps >= max_steps:
            status, message = 2, "step budget reached"
    return Solution(t, y, nfev[0], status, message, steps)
