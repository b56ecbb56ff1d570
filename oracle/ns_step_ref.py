"""ORACLE (test infrastructure only) -- ctypes wrapper of ns_step_ref.c.

numpy float32 in/out; plane convention of the reference (see ns_step_ref.c).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "lib", "libns_ref.so")
_dll = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _lib():
    global _dll
    if _dll is None:
        if not os.path.exists(_LIB):
            build()
        _dll = ctypes.CDLL(_LIB)
        P, I, L, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
        _dll.ns_ref_gradient.argtypes = [P, L, P, P, I, I, I, F]
        _dll.ns_ref_cip.argtypes = [P, L, P, P, P, P, L, I, I, I, F, F]
        _dll.ns_ref_vel_update.argtypes = [P, P, P, P, I, I, I, F]
        _dll.ns_ref_pressure.argtypes = [P, P, P, I, I, I, F, F]
        _dll.ns_ref_update_density.argtypes = [P, P, P, I, I, I, F, F]
        _dll.ns_ref_update_velocity.argtypes = [P, P, P, I, I, I, F, F, I]
        _dll.ns_ref_advect.argtypes = [P, P, P, P, P, I, I, I, F]
    return _dll


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _geo(a):
    B, _, nx, ny = a.shape
    return B, nx, ny


def update_density(dens, vel, dt, dx):
    dens, vel = _f32(dens), _f32(vel)
    out = np.empty_like(dens)
    B, nx, ny = _geo(dens)
    _lib().ns_ref_update_density(_p(dens), _p(vel), _p(out), B, nx, ny, dt, dx)
    return out


def update_velocity(vel, pres, dt, dx, compat=True):
    vel, pres = _f32(vel), _f32(pres)
    out = np.empty_like(vel)
    B, nx, ny = _geo(vel)
    _lib().ns_ref_update_velocity(_p(vel), _p(pres), _p(out), B, nx, ny, dt, dx, int(compat))
    return out


def update_pressure(pres, vel, dt, dx):
    pres, vel = _f32(pres), _f32(vel)
    out = np.empty_like(pres)
    B, nx, ny = _geo(pres)
    _lib().ns_ref_pressure(_p(pres), _p(vel), _p(out), B, nx, ny, dt, dx)
    return out


def gradient(f, dx):
    f = _f32(f)
    B, nx, ny = _geo(f)
    fx, fy = np.empty_like(f), np.empty_like(f)
    _lib().ns_ref_gradient(_p(f), nx * ny, _p(fx), _p(fy), B, nx, ny, dx)
    return fx, fy


def full_step(dens, vel, pres, dt, dx, compat=True):
    """pinn_kalman/simulator.py:55-57 order: velocity, pressure(new vel), density(new vel)."""
    v1 = update_velocity(vel, pres, dt, dx, compat)
    p1 = update_pressure(pres, v1, dt, dx)
    d1 = update_density(dens, v1, dt, dx)
    return d1, v1, p1
