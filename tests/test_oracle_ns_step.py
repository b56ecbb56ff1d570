"""CPU: analytic known-answer tests pinning the C restatement of ns_step (no runnable reference:
the reference op is a CUDA-only extension)."""
import numpy as np
import pytest

from oracle import ns_step_ref as ns

DT, DX = 0.0025, 0.005


def _linear(B, nx, ny, a, b, c=0.0):
    x = np.arange(nx, dtype=np.float32) * DX
    y = np.arange(ny, dtype=np.float32) * DX
    f = (a * x[None, :] + b * y[:, None] + c).astype(np.float32)  # plane[y, x]
    return np.broadcast_to(f.reshape(1, 1, ny, nx), (B, 1, ny, nx)).copy()


def _as_ref_layout(a):
    # reference indexes field[y * nx + x] with nx = size(2): a [B,1,ny,nx] C-array has exactly
    # that memory; present it with shape [B, 1, nx, ny] as the reference tensors would be
    B, C, ny, nx = a.shape
    return a.reshape(B, C, nx, ny)


def test_gradient_of_linear_field_is_exact():
    f = _as_ref_layout(_linear(2, 9, 7, 3.0, -2.0))
    fx, fy = ns.gradient(f, DX)
    np.testing.assert_allclose(fx, 3.0, rtol=2e-3)
    np.testing.assert_allclose(fy, -2.0, rtol=2e-3)


def test_cip_keeps_constant_field_and_translates_linear_field():
    B, n = 2, 12
    rng = np.random.default_rng(0)
    vel = (rng.uniform(0.05, 0.5, (B, 2, n, n)) * rng.choice([-1, 1], (B, 2, n, n))).astype(np.float32)
    const = np.full((B, 1, n, n), 1.25, np.float32)
    np.testing.assert_array_equal(ns.update_density(const, vel, DT, DX), const)
    lin = _as_ref_layout(_linear(B, n, n, 2.0, 0.5, 1.0))
    out = ns.update_density(lin, vel, DT, DX)
    u = vel[:, 0].reshape(B, n, n)
    v = vel[:, 1].reshape(B, n, n)
    exact = lin[:, 0].reshape(B, n, n) - (2.0 * u + 0.5 * v) * DT
    inner = (slice(None), slice(2, -2), slice(2, -2))
    np.testing.assert_allclose(out[:, 0].reshape(B, n, n)[inner], exact[inner], rtol=0, atol=2e-6)


def test_pressure_update_of_rest_state():
    B, n = 3, 8
    p = np.full((B, 1, n, n), 0.7, np.float32)
    vel = np.zeros((B, 2, n, n), np.float32)
    np.testing.assert_allclose(ns.update_pressure(p, vel, DT, DX), 0.7, rtol=1e-7)


def test_zero_velocity_gives_nan_like_the_reference():
    """CIP divides by sign(u) * dx^3 (op/ns_step_kernel.cu:137-146)."""
    B, n = 1, 6
    f = np.random.default_rng(1).standard_normal((B, 1, n, n)).astype(np.float32)
    vel = np.zeros((B, 2, n, n), np.float32)
    assert np.isnan(ns.update_density(f, vel, DT, DX)).any()


def test_unbind_quirk_only_matters_for_batch_two_or_more():
    rng = np.random.default_rng(2)
    n = 10
    for B, same in ((1, True), (3, False)):
        vel = (rng.uniform(0.05, 0.5, (B, 2, n, n)) * rng.choice([-1, 1], (B, 2, n, n))).astype(np.float32)
        p = rng.normal(0, 0.01, (B, 1, n, n)).astype(np.float32)
        a = ns.update_velocity(vel, p, DT, DX, compat=True)
        b = ns.update_velocity(vel, p, DT, DX, compat=False)
        assert np.array_equal(a, b) == same
        if not same:  # sample 0's u plane is the same in both modes (plane 0 of vel_n)
            np.testing.assert_array_equal(a[0, 0], b[0, 0])
