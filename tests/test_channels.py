"""op.channels (CPU): cat / swap_scale equal the torch ops they replace, and their first,
second and third derivatives equal torch's (float64 gradcheck / gradgradcheck plus an explicit
third-order comparison), with every order one cat / split / swap op (the PINN residual
differentiates FlowNet three times, reference pinn.py:72-111)."""
import pytest
import torch

from op import channels


def _inputs(shapes, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(*s, generator=g, dtype=torch.float64, requires_grad=True) for s in shapes]


def test_cat_values_and_gradients_match_torch():
    xs = _inputs([(2, 3, 4, 5), (2, 1, 4, 5), (2, 2, 4, 5)], 0)
    assert torch.equal(channels.cat(xs, 1), torch.cat(xs, 1))
    assert torch.autograd.gradcheck(lambda *a: channels.cat(a, 1), xs)
    assert torch.autograd.gradgradcheck(lambda *a: channels.cat(a, 1), xs)
    assert torch.equal(channels.cat(xs[:1], 1), xs[0])


def test_swap_scale_values_and_gradients_match_torch():
    u, = _inputs([(3, 2, 4, 6)], 1)
    ref = torch.cat([u[:, 1:2] / 1.5, u[:, 0:1] / 2.5], 1)
    assert torch.equal(channels.swap_scale(u, 1.5, 2.5), ref)
    assert torch.autograd.gradcheck(lambda a: channels.swap_scale(a, 1.5, 2.5), (u,))
    assert torch.autograd.gradgradcheck(lambda a: channels.swap_scale(a, 1.5, 2.5), (u,))


def _third_order(f, xs, w):
    """d/dx of sum(w * d/dx(sum(d/dx(sum(f(x)^3)))^2)): three nested differentiations"""
    y = (f(*xs) ** 3).sum()
    g1 = torch.autograd.grad(y, xs, create_graph=True)
    z = sum(((gi * wi) ** 2).sum() for gi, wi in zip(g1, w))
    g2 = torch.autograd.grad(z, xs, create_graph=True)
    q = sum((gi.sin() * wi).sum() for gi, wi in zip(g2, w))
    return torch.autograd.grad(q, xs)


def test_third_derivatives_match_torch():
    xs = _inputs([(2, 3, 3, 3), (2, 2, 3, 3)], 2)
    w = [torch.randn_like(x) for x in xs]
    a = _third_order(lambda *t: channels.cat(t, 1) * torch.arange(5.0, dtype=torch.float64).view(1, 5, 1, 1), xs, w)
    b = _third_order(lambda *t: torch.cat(t, 1) * torch.arange(5.0, dtype=torch.float64).view(1, 5, 1, 1), xs, w)
    for p, q in zip(a, b):
        torch.testing.assert_close(p, q, rtol=1e-12, atol=1e-12)
    u, = _inputs([(2, 2, 3, 4)], 3)
    wu = [torch.randn_like(u)]
    a = _third_order(lambda t: channels.swap_scale(t, 0.7, 1.3), [u], wu)
    b = _third_order(lambda t: torch.cat([t[:, 1:2] / 0.7, t[:, 0:1] / 1.3], 1), [u], wu)
    torch.testing.assert_close(a[0], b[0], rtol=1e-12, atol=1e-12)


def test_sum2x2_adjoint_pair_cpu_f64():
    """op.conv._sum2x2 (the 2 x 2 block sum behind conv3x3_up2's input gradient) on the host
    path: first and second derivatives by gradcheck; its adjoint is the nearest upsample."""
    from op.conv import _sum2x2
    x = torch.randn(2, 3, 4, 6, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(_sum2x2, (x,))
    assert torch.autograd.gradgradcheck(_sum2x2, (x,))
    y = _sum2x2(x)
    assert torch.allclose(y, x.reshape(2, 3, 2, 2, 3, 2).sum((3, 5)))


@pytest.mark.parametrize("used", [(0,), (1, 3), (0, 1, 2, 3), (2,)])
def test_split_backward_with_unused_pieces(used):
    """channels.split whose pieces are only partly used (PINN.forward_residual_copies reads
    copy 0 of most splits): the backward fills the unused pieces' rows with zeros in one op
    (_PadCat) -- same gradient as torch.split, and differentiable again (gradcheck /
    gradgradcheck in float64)."""
    torch.manual_seed(0)
    x = torch.randn(8, 3, 2, dtype=torch.float64, requires_grad=True)

    def f(split):
        def g(x):
            ps = split(x * 1.5)
            return sum(((ps[i] ** 2) * (i + 1)).sum() for i in used)
        return g

    ours = f(lambda t: channels.split(t, (2, 2, 2, 2), 0))
    ref = f(lambda t: torch.split(t, [2, 2, 2, 2], 0))
    g1, = torch.autograd.grad(ours(x), x)
    g2, = torch.autograd.grad(ref(x), x)
    assert torch.equal(g1, g2)
    assert torch.autograd.gradcheck(ours, (x,))
    assert torch.autograd.gradgradcheck(ours, (x,))
