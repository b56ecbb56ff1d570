"""CPU tests of the PINN path: correlation oracle known answers, PINN construction and
state-dict layout, the gather-form inpainting operator (no GPU needed)."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import correlation_ref as cr


def _brute(first, second, s):
    B, C, H, W = first.shape
    Ho, Wo = -(-H // s), -(-W // s)
    out = np.zeros((B, 49, Ho, Wo))
    for b in range(B):
        for d in range(49):
            dy, dx = (d // 7 - 3) * s, (d % 7 - 3) * s
            for oy in range(Ho):
                for ox in range(Wo):
                    y, x = oy * s, ox * s
                    if 0 <= y + dy < H and 0 <= x + dx < W:
                        out[b, d, oy, ox] = (first[b, :, y, x].astype(np.float64)
                                             * second[b, :, y + dy, x + dx]).mean()
    return out


@pytest.mark.parametrize("shape,s", [((2, 3, 7, 6), 1), ((1, 4, 9, 9), 2), ((1, 2, 5, 11), 3)])
def test_correlation_oracle_known_answers(shape, s):
    rng = np.random.default_rng(0)
    a = rng.standard_normal(shape).astype(np.float32)
    b = rng.standard_normal(shape).astype(np.float32)
    out = cr.forward(a, b, s)
    np.testing.assert_allclose(out, _brute(a, b, s), rtol=1e-6, atol=1e-6)
    # all-ones: the value is the fraction of the displaced window inside the image
    ones = np.ones(shape, np.float32)
    o1 = cr.forward(ones, ones, s)
    assert set(np.unique(o1)) <= {0.0, 1.0}
    assert o1[:, 24].min() == 1.0  # zero displacement always inside


@pytest.mark.parametrize("s", [1, 2])
def test_correlation_oracle_grads_are_the_adjoint(s):
    """out is bilinear in (first, second): <g, out> = <grad_first, first> = <grad_second, second>."""
    rng = np.random.default_rng(1)
    a = rng.standard_normal((2, 3, 8, 7)).astype(np.float32)
    b = rng.standard_normal((2, 3, 8, 7)).astype(np.float32)
    out = cr.forward(a, b, s)
    g = rng.standard_normal(out.shape).astype(np.float32)
    gf, gs = cr.backward(a, b, g, s)
    lhs = (out.astype(np.float64) * g).sum()
    assert abs(lhs - (gf.astype(np.float64) * a).sum()) < 1e-4 * max(1, abs(lhs))
    assert abs(lhs - (gs.astype(np.float64) * b).sum()) < 1e-4 * max(1, abs(lhs))


def _pinn_cfg():
    from configs.pinn import pinn_pde
    c = pinn_pde.get_config()
    c.device = torch.device("cpu")
    return c


def test_pinn_parameter_counts_match_reference():
    """FlowNet 2.488 M + PressureNet 7.539 M at pinn_pde."""
    from pinn_kalman.pinn import PINN
    m = PINN(_pinn_cfg())
    assert sum(p.numel() for p in m.flownet.parameters()) == 2487622
    assert sum(p.numel() for p in m.pressurenet.parameters()) == 7538936
    assert all(not k.startswith("mask") for k in m.state_dict())


def test_pinn_seeded_weights_reproduce_reference_fixture():
    """The seeded construction recipe of the fixture generator yields the reference's
    weights bit for bit (same module order and init) -- the GPU tests rely on it."""
    from conftest import build_pinn_weights, sample_idx, small_config
    from configs.pinn import pinn_pde
    from pinn_kalman.pinn import PINN
    d = load_golden("pinn_fwd.npz")
    m = build_pinn_weights(PINN, small_config(pinn_pde.get_config))
    sd = m.state_dict()
    keys = [k[6:] for k in d.files if k.startswith("sdsub:")]
    assert sorted(keys) == sorted(sd.keys())
    for k in keys:
        v = sd[k].reshape(-1).numpy()
        np.testing.assert_array_equal(v[sample_idx(v.size)], d["sdsub:" + k])


def test_inpaint_operator_gather_matches_dense_selection():
    from inverse.operators import InpaintOperator, random_mask_source
    c = _pinn_cfg()
    c.data.image_size = 8
    c.training.batch_size = 3
    masks = random_mask_source(c, n=4, generator=torch.Generator().manual_seed(0))
    assert abs(float(masks[0].mean()) - 0.9) < 0.1
    op = InpaintOperator(mask=masks)
    x = torch.randn(3, 1, 8, 8)
    np.testing.assert_array_equal((op(x) - masks[0] * x).numpy(), 0)
    y = op(x, keep_shape=False)
    # dense form of the reference: rows of diag(mask) with a 1, transposed (operators.py:170-172)
    m = masks[0][0, 0].flatten()
    pL = torch.diag(m)[torch.where(torch.diag(m).sum(1) == 1)[0]].T
    dense = x.reshape(3, 1, 1, 64) @ pL
    np.testing.assert_array_equal(y.numpy(), dense.reshape(3, 1, -1).numpy())
    back = op.transpose(y, x.shape)
    np.testing.assert_array_equal(back.numpy(), (masks[0] * x).numpy())
    op.next()
    assert op.mask is masks[1]


def test_batched_timestep_embeddings_equal_per_level_calls():
    """layers.get_timestep_embeddings (FlowNet's per-level embeddings as one product / sin / cos)
    == get_timestep_embedding per level as the reference computes it (models/layers.py:500-514),
    bit for bit, odd and one-channel dims included; and the same gradient w.r.t. t."""
    import math

    import models.layers as L
    t = torch.tensor([300., 512., 899., 301.], requires_grad=True)
    dims = [1, 16, 32, 64, 96, 7]
    got = L.get_timestep_embeddings(t, dims)
    ref = []
    for d in dims:
        half = d // 2
        rate = math.log(10000) / (half - 1)
        fr = torch.exp(torch.arange(half, dtype=torch.float32) * -rate)
        arg = t.float()[:, None] * fr[None, :]
        r = torch.cat([torch.sin(arg), torch.cos(arg)], 1)
        if d % 2:
            r = torch.nn.functional.pad(r, (0, 1))
        ref.append(r)
        assert torch.equal(L.get_timestep_embedding(t, d), r)
    w = [torch.randn(r.shape, generator=torch.Generator().manual_seed(i)) for i, r in enumerate(ref)]
    for a, b in zip(got, ref):
        assert a.shape == b.shape and torch.equal(a, b)
    ga = torch.autograd.grad(sum((a * v).sum() for a, v in zip(got, w)), t)[0]
    gb = torch.autograd.grad(sum((b * v).sum() for b, v in zip(ref, w)), t)[0]
    torch.testing.assert_close(ga, gb, rtol=1e-6, atol=1e-6)
