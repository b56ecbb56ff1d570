"""CPU checks of the stencil-residual and UKF-dynamics oracles (oracle/pinn_fd_ref.py) and of
the build's patch / unpatch (pure tensor reshapes, run on CPU here)."""
import numpy as np
import torch

from oracle import pinn_fd_ref


def test_float64_stencil_matches_the_c_oracle():
    rng = np.random.default_rng(0)
    # square planes: the reference's plane convention f[y * nx + x] takes nx = size(2) for
    # the contiguous axis (op/ns_step_kernel.cu:30-37), i.e. assumes H == W
    f = rng.standard_normal((2, 1, 23, 23)).astype(np.float32)
    assert pinn_fd_ref.check_stencil_matches_c(f, 0.05) < 1e-6


def test_fd_residual_of_a_known_field():
    """u = x, v = -y (divergence-free, steady): u u_x + v u_y = x, mass residual 0; with
    p = 0, u_t = v_t = 0 the residual mse is mean(x^2) + mean(y^2) (exact stencils on
    linear fields, zero second derivatives)."""
    n, h = 16, 0.1
    xs = np.arange(n) * h
    X, Y = np.meshgrid(xs, xs)
    u = X[None, None]
    v = -Y[None, None]
    zero = np.zeros_like(u)
    got = pinn_fd_ref.fd_residual_mse(u, v, zero, np.zeros(1), np.zeros(1), h, 1e7)
    # (h enters as float32, as the kernels take it)
    assert abs(got - ((X ** 2).mean() + (Y ** 2).mean())) < 1e-6


def test_patch_unpatch_match_the_oracle_and_invert():
    from pinn_kalman.ukf_utils import patch, unpatch
    rng = np.random.default_rng(1)
    x = rng.standard_normal((3, 4, 16, 16)).astype(np.float32)
    rows = patch(torch.from_numpy(x), 8).numpy()
    np.testing.assert_array_equal(rows, pinn_fd_ref.patch(x, 8))
    back = unpatch(torch.from_numpy(rows), 8, 16, 4).numpy()
    np.testing.assert_array_equal(back, x)
    np.testing.assert_array_equal(pinn_fd_ref.unpatch(rows, 8, 16, 4), x)
