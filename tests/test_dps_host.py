"""CPU tests of the inverse-problem path: the device RK solver reproduces scipy's
solve_ivp (the reference's solver) step for step, the sharded-norm hook, LOBSVSDE."""
import numpy as np
import pytest
import torch
from scipy.integrate import solve_ivp


def _system(n=40, seed=0):
    rng = np.random.default_rng(seed)
    W = rng.standard_normal((n, n)) / np.sqrt(n)
    y0 = rng.standard_normal(n)
    Wt = torch.tensor(W)
    return (lambda t, y: np.tanh(W @ y) * (1 + t) - 0.5 * y,
            lambda t, y: torch.tanh(Wt @ y) * (1 + t) - 0.5 * y, y0)


@pytest.mark.parametrize("method", ["RK45", "RK23"])
@pytest.mark.parametrize("tol", [1e-3, 1e-6])
def test_rk_solver_matches_scipy(method, tol):
    from inverse.ode import solve_ivp_rk
    fnp, ft, y0 = _system()
    ref = solve_ivp(fnp, (1.0, 1e-3), y0, method=method, rtol=tol, atol=tol)
    out = solve_ivp_rk(ft, (1.0, 1e-3), torch.tensor(y0), method=method, rtol=tol, atol=tol)
    assert out.nfev == ref.nfev and out.n_steps == len(ref.t) - 1 and out.status == ref.status
    np.testing.assert_allclose(out.y.numpy(), ref.y[:, -1], rtol=0, atol=1e-12)


def _shard_worker(rank, world, port, q):
    import os
    import sys
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import dist
    from inverse.conditional_sampling import _reduce_sumsq_fn
    from inverse.ode import solve_ivp_rk
    ctx = dist.init_from_env(backend="gloo")
    y0, a = _decay_system()
    off, n = dist.shard(64, ctx)
    red, w = _reduce_sumsq_fn(ctx)
    sl = slice(off, off + n)
    out = solve_ivp_rk(lambda t, y: -a[sl] * y * (1 + t) + 0.1 * torch.sin(y), (1.0, 1e-3),
                       y0[sl], rtol=1e-6, atol=1e-6, reduce_sumsq=red, n_global=64)
    q.put((rank, out.nfev, out.n_steps, out.y.tolist()))
    torch.distributed.destroy_process_group()


def _decay_system():
    rng = np.random.default_rng(1)
    return torch.tensor(rng.standard_normal(64)), torch.tensor(rng.uniform(0.5, 20.0, 64))


def test_rk_solver_batch_sharded_gloo_world2_matches_single_process():
    """Two ranks each integrate half of the state with the all-reduced RMS norms: the
    accepted steps, nfev and final state equal the single-process solve."""
    import multiprocessing as mp
    import os
    from inverse.ode import solve_ivp_rk
    y0, a = _decay_system()
    full = solve_ivp_rk(lambda t, y: -a * y * (1 + t) + 0.1 * torch.sin(y), (1.0, 1e-3), y0,
                        rtol=1e-6, atol=1e-6)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000
    ps = [ctx.Process(target=_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for rank, nfev, steps, y in res:
        assert nfev == full.nfev and steps == full.n_steps
    y = np.concatenate([res[0][3], res[1][3]])
    np.testing.assert_allclose(y, full.y.numpy(), rtol=0, atol=1e-12)


def test_lobsvsde_observe_sampling():
    import sde_lib
    from inverse.operators import InpaintOperator
    mask = (torch.rand(1, 1, 8, 8, generator=torch.Generator().manual_seed(0)) > 0.5).float()
    mask = mask.expand(3, 1, 8, 8).contiguous()
    op = InpaintOperator(mask=[mask])
    x0 = torch.randn(3, 1, 8, 8)
    y0 = op(x0, keep_shape=False)
    sde = sde_lib.VPSDE()
    obs = sde_lib.LOBSVSDE(sde, y0, op)
    t = torch.tensor([0.1, 0.5, 0.9])
    z = torch.randn(3, 1, 8, 8)
    a, b = sde.marginal_coef(t)
    expect = a[:, None, None] * y0 + b[:, None, None] * op(z, keep_shape=False)
    assert torch.equal(obs.observe_sampling(z, t), expect)
    assert obs.T == 1 and obs.N == sde.N
