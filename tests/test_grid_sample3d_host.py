"""CPU pinning of the 3-D grid_sample double-backward oracle (oracle/grid_sample_ref.grad3,
a restatement of the reference's op/grid_sample_kernel.cu:212-533): its outputs are the
gradients of L = <g2_inp, grad_input> + <g2_grid, grad_grid> of ATen's own first backward
(aten::grid_sampler_3d_backward, which the reference calls), checked by float64 central
differences along random directions."""
import pytest
import torch

from oracle import grid_sample_ref as gs


def _L(gout, inp, grid, g2i, g2g, pm):
    gi, gg = gs.bwd3(gout, inp, grid, pm, True)
    return (g2i * gi).sum() + (g2g * gg).sum()


@pytest.mark.parametrize("pm", [0, 1])
def test_grad3_oracle_is_the_derivative_of_the_first_backward(pm):
    g = torch.Generator().manual_seed(7 + pm)
    N, C, D, H, W, Do, Ho, Wo = 2, 3, 4, 5, 6, 3, 2, 4
    d = torch.float64
    inp = torch.randn(N, C, D, H, W, generator=g, dtype=d)
    grid = torch.rand(N, Do, Ho, Wo, 3, generator=g, dtype=d) * 2.2 - 1.1
    gout = torch.randn(N, C, Do, Ho, Wo, generator=g, dtype=d)
    g2i = torch.randn(inp.shape, generator=g, dtype=d)
    g2g = torch.randn(grid.shape, generator=g, dtype=d)
    ggo, gin, ggrid = gs.grad3(g2i, g2g, gout, inp, grid, pm, True)
    eps = 1e-6
    for k, (arg, grad) in enumerate(((gout, ggo), (inp, gin), (grid, ggrid))):
        for _ in range(3):
            dirn = torch.randn(arg.shape, generator=g, dtype=d)
            args = [gout, inp, grid]
            args[k] = arg + eps * dirn
            lp = _L(*args, g2i, g2g, pm)
            args[k] = arg - eps * dirn
            lm = _L(*args, g2i, g2g, pm)
            fd = (lp - lm) / (2 * eps)
            an = (grad * dirn).sum()
            assert abs(fd - an) <= 1e-6 * max(1.0, abs(an)), (k, float(fd), float(an))
