"""GPU parity of the native ops (HIP kernels via the C ABI) against the oracle / fixtures."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import load_golden
from oracle import fused_act_ref, grid_sample_ref, ns_step_ref
from oracle.upfirdn2d_ref import upfirdn2d_np

pytestmark = pytest.mark.gpu


# ------------------------------------------------------------------ upfirdn2d
def _golden_cases():
    d = load_golden("upfirdn2d.npz")
    out = []
    for c in range(int(d["n_cases"])):
        p = d[f"c{c}_params"]
        out.append((d[f"c{c}_x"], d[f"c{c}_k"], (int(p[0]), int(p[1])), (int(p[2]), int(p[3])),
                    tuple(int(v) for v in p[4:]), d[f"c{c}_y"], d[f"c{c}_g"], d[f"c{c}_gx"]))
    return out


@pytest.mark.parametrize("case", range(12))
def test_upfirdn2d_matches_reference_fixture_fwd_and_bwd(hip, case):
    from op.upfirdn2d import upfirdn2d_xy
    x, k, up, down, pad, y, g, gx = _golden_cases()[case]
    xt = torch.tensor(x, device=hip, requires_grad=True)
    out = upfirdn2d_xy(xt, torch.tensor(k, device=hip), up, down, pad)
    tol = 2e-6 * max(1.0, float(np.abs(y).max()))
    np.testing.assert_allclose(out.detach().cpu().numpy(), y, rtol=0, atol=tol)
    (gin,) = torch.autograd.grad(out, xt, torch.tensor(g, device=hip))
    np.testing.assert_allclose(gin.cpu().numpy(), gx, rtol=0,
                               atol=2e-6 * max(1.0, float(np.abs(gx).max())))


@pytest.mark.parametrize("shape,up,down,pad,gain", [
    ((4, 64, 64, 64), 1, 2, (1, 1), 1), ((4, 64, 32, 32), 2, 1, (2, 1), 4),
    ((4, 32, 64, 64), 1, 1, (2, 2), 1), ((2, 16, 16, 16), 2, 1, (2, 1), 4),
    ((2, 16, 32, 32), 1, 2, (1, 1), 1), ((3, 5, 37, 23), 1, 2, (1, 1), 1)])
def test_upfirdn2d_ncsnpp_modes_vs_oracle(hip, shape, up, down, pad, gain):
    from op import upfirdn2d
    rng = np.random.default_rng(0)
    x = rng.standard_normal(shape).astype(np.float32)
    k = np.outer([1, 3, 3, 1], [1, 3, 3, 1]).astype(np.float32) / 64 * gain
    y = upfirdn2d(torch.tensor(x, device=hip), torch.tensor(k, device=hip), up=up, down=down,
                  pad=pad).cpu().numpy()
    ref = upfirdn2d_np(x.astype(np.float64), k, (up, up), (down, down),
                       (pad[0], pad[1], pad[0], pad[1]))
    np.testing.assert_allclose(y, ref, rtol=0, atol=2e-6)


@pytest.mark.parametrize("shape", [(64, 128, 128, 128), (64, 256, 64, 64), (24, 512, 128, 128),
                                   (2, 8, 38, 64), (5, 3, 64, 256)])
def test_upfirdn2d_down2_row_rolling_strips(hip, shape):
    """down2 pad(1,1) on the row-rolling kernel at every strip form it takes: strips of 8, 4 and
    16 output rows held in registers (the 8(d) shapes and a bigger one), a height the strip does
    not divide (per-row stores) and a 64-lane segment; vs the same FIR as a stride-2 conv on the
    flipped taps (F.conv2d, fp32)."""
    from op import upfirdn2d
    g = torch.Generator(device=hip).manual_seed(sum(shape))
    x = torch.randn(*shape, device=hip, generator=g)
    k = torch.tensor(np.outer([1, 3, 3, 1], [1, 3, 3, 1]) / 64.0, dtype=torch.float32, device=hip)
    y = upfirdn2d(x, k, down=2, pad=(1, 1))
    N, C, H, W = shape
    ref = F.conv2d(x.view(N * C, 1, H, W), k.flip(0, 1)[None, None], stride=2, padding=1)
    assert y.shape == (N, C, H // 2, W // 2)
    assert (y - ref.view_as(y)).abs().max().item() <= 2e-6


def test_upfirdn2d_second_order_gradcheck_f64(hip):
    from op import upfirdn2d
    k = torch.tensor(np.outer([1, 3, 3, 1], [1, 3, 3, 1]) / 64.0, device=hip)
    x = torch.randn(1, 2, 6, 6, dtype=torch.float64, device=hip, requires_grad=True)
    for up, down, pad in [(1, 2, (1, 1)), (2, 1, (2, 1))]:
        f = lambda t: upfirdn2d(t, k * (4 if up == 2 else 1), up=up, down=down, pad=pad)
        assert torch.autograd.gradcheck(f, (x,))
        assert torch.autograd.gradgradcheck(f, (x,))


def test_upfirdn2d_large_plane_count_and_empty_batch(hip):
    from op import upfirdn2d
    k = torch.ones(4, 4, device=hip) / 16
    x = torch.randn(70000, 1, 4, 4, device=hip)  # > 65535 planes: 1-D grid mapping
    y = upfirdn2d(x, k, down=2, pad=(1, 1))
    ref = upfirdn2d_np(x[:5].cpu().numpy(), k.cpu().numpy(), (1, 1), (2, 2), (1, 1, 1, 1))
    np.testing.assert_allclose(y[:5].cpu().numpy(), ref, atol=1e-6)
    assert upfirdn2d(torch.zeros(0, 3, 8, 8, device=hip), k, down=2, pad=(1, 1)).shape == (0, 3, 4, 4)


# ------------------------------------------------------------------ fused_bias_act
def test_fused_leaky_relu_matches_fixture_and_oracle(hip):
    from op import fused_leaky_relu
    d = load_golden("fused_lrelu.npz")
    y = fused_leaky_relu(torch.tensor(d["x"], device=hip), torch.tensor(d["b"], device=hip))
    np.testing.assert_allclose(y.cpu().numpy(), d["y"], rtol=1e-6, atol=1e-6)
    x = np.random.default_rng(3).standard_normal((2, 6, 5, 5)).astype(np.float32)
    b = np.random.default_rng(4).standard_normal(6).astype(np.float32)
    y = fused_leaky_relu(torch.tensor(x, device=hip), torch.tensor(b, device=hip), 0.1, 1.7)
    np.testing.assert_allclose(y.cpu().numpy(), fused_act_ref.fused_bias_act(x, b, None, 3, 0, 0.1, 1.7),
                               rtol=1e-6, atol=1e-6)


def test_fused_leaky_relu_grads_f64(hip):
    from op import fused_leaky_relu
    x = torch.randn(2, 3, 4, 4, dtype=torch.float64, device=hip, requires_grad=True)
    b = torch.randn(3, dtype=torch.float64, device=hip, requires_grad=True)
    f = lambda a, c: fused_leaky_relu(a, c, 0.2, 2 ** 0.5)
    assert torch.autograd.gradcheck(f, (x, b))
    assert torch.autograd.gradgradcheck(f, (x, b))


@pytest.mark.parametrize("shape", [(3, 5, 7, 9), (4, 8, 16, 16)])  # scalar / float4 kernel
@pytest.mark.parametrize("slope", [0.1, 0.01])
def test_native_leaky_relu_bit_identical_to_aten_to_third_order(hip, slope, shape):
    """op.fused_act.leaky_relu (FlowNet's activation on the native kernel): forward, first,
    second and third derivatives bit-identical to F.leaky_relu under autograd, and f64
    gradcheck / gradgradcheck.  (The mask's derivative is not materialized: a derivative whose
    only path is through it has no graph here, where aten builds one of zeros.)"""
    import torch.nn.functional as F
    from op.fused_act import leaky_relu
    g = torch.Generator().manual_seed(5)
    x0 = torch.randn(*shape, generator=g)
    x0[0, 0, 0, :3] = 0.0  # the x == 0 boundary takes the slope branch in both
    w = torch.randn(*shape, generator=g).to(hip)

    def derivs(fn):
        x = x0.to(hip).requires_grad_()
        y = fn(x)
        (d1,) = torch.autograd.grad((y * w).sum(), x, create_graph=True)
        (d2,) = torch.autograd.grad((d1 * y * y).sum(), x, create_graph=True)
        (d3,) = torch.autograd.grad((d2 * y).sum(), x)
        return [t.detach() for t in (y, d1, d2, d3)]
    for a, b in zip(derivs(lambda v: leaky_relu(v, slope)), derivs(lambda v: F.leaky_relu(v, slope))):
        assert torch.equal(a, b)
    x = torch.randn(2, 3, 4, 4, dtype=torch.float64, device=hip, requires_grad=True)
    assert torch.autograd.gradcheck(lambda v: leaky_relu(v, slope), (x,))
    assert torch.autograd.gradgradcheck(lambda v: leaky_relu(v, slope), (x,))


@pytest.mark.parametrize("shape", [(3, 2, 16, 20), (2, 2, 5, 7), (64, 2, 32, 32)])
def test_swap_scale_native_bit_identical_to_aten(hip, shape):
    """op.channels.swap_scale (FlowNet's project: torch.cat([u[:, 1:2] / c0, u[:, 0:1] / c1], 1))
    on the native kernel (csrc/channels.hip; float4 and scalar paths) == aten bit for bit, in
    the forward and through three derivative orders."""
    from op import channels
    g = torch.Generator().manual_seed(shape[0])
    u0 = torch.randn(*shape, generator=g).to(hip)
    c0, c1 = (shape[2] - 1.0) / 2.0, (shape[3] - 1.0) / 2.0

    def derivs(fn):
        u = u0.clone().requires_grad_()
        y = fn(u)
        w = torch.sin(torch.arange(y.numel(), device=hip, dtype=torch.float32)).view_as(y)
        (d1,) = torch.autograd.grad((y * w).sum(), u, create_graph=True)
        return y.detach(), d1.detach()

    got = derivs(lambda u: channels.swap_scale(u * u, c0, c1))
    ref = derivs(lambda u: torch.cat([(u * u)[:, 1:2] / c0, (u * u)[:, 0:1] / c1], 1))
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    # the adjoint's own backward (third order in the PINN residual) is the same kernel
    u = u0.clone().requires_grad_()
    y = channels.swap_scale(u, c0, c1)
    (g1,) = torch.autograd.grad(y, u, torch.ones_like(y), create_graph=True)
    assert torch.equal(g1[:, 0], torch.ones_like(g1[:, 0]) / c1)
    assert torch.equal(g1[:, 1], torch.ones_like(g1[:, 1]) / c0)
    # channels-last input (the gradients coming back through project's NHWC grid view): run in
    # that layout, same bits
    ucl = u0.permute(0, 2, 3, 1).contiguous().permute(0, 3, 1, 2)
    assert not ucl.is_contiguous()
    with torch.no_grad():
        y = channels._SwapScale.apply(ucl, c0, c1)
    assert y.stride() == ucl.stride()
    assert torch.equal(y, torch.cat([ucl[:, 1:2] / c0, ucl[:, 0:1] / c1], 1))


@pytest.mark.parametrize("shape", [(2, 3, 8, 12), (3, 5, 6, 10), (1, 2, 4, 6)])
def test_sum2x2_native_vs_block_sum(hip, shape):
    """the 2 x 2 block sum behind conv3x3_up2's input gradient (csrc/channels.hip; float2 and
    scalar output paths) vs the reshape-sum it replaces (1e-6 of max|ref|: a different
    summation order), and its adjoint is the nearest upsample (gradient check in float32)."""
    from op.conv import _sum2x2
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(*shape, generator=g).to(hip)
    N, C, H2, W2 = shape
    ref = x.reshape(N, C, H2 // 2, 2, W2 // 2, 2).sum((3, 5))
    got = _sum2x2(x)
    assert got.shape == ref.shape
    assert (got - ref).abs().max().item() <= 1e-6 * max(1.0, ref.abs().max().item())
    xr = x.clone().requires_grad_()
    gy = torch.randn(ref.shape, generator=g).to(hip)
    (gx,) = torch.autograd.grad(_sum2x2(xr), xr, gy)
    assert torch.equal(gx, torch.nn.functional.interpolate(gy, scale_factor=2, mode="nearest"))


# ------------------------------------------------------------------ GroupNorm + SiLU
@pytest.mark.parametrize("N,C,H,G", [(2, 64, 16, 16), (3, 128, 32, 32), (2, 256, 64, 32),
                                      (2, 384, 64, 32), (1, 8, 5, 2), (2, 32, 128, 8),
                                      (1, 16, 256, 4), (1, 64, 151, 4)])
@pytest.mark.parametrize("act", [0, 1])
def test_group_norm_act_fwd_bwd_vs_torch(hip, N, C, H, G, act):
    from op.norm_act import group_norm_act_f
    torch.manual_seed(0)
    x = torch.randn(N, C, H, H) * 2 + 0.5
    bnc = torch.randn(N, C)
    w = torch.randn(C)
    b = torch.randn(C)
    dy = torch.randn(N, C, H, H)
    xs = [t.clone().requires_grad_(True) for t in (x, bnc, w, b)]
    ref = F.group_norm(xs[0] + xs[1][:, :, None, None], G, xs[2], xs[3], eps=1e-6)
    if act:
        ref = F.silu(ref)
    ref.backward(dy)
    xg = [t.to(hip).requires_grad_(True) for t in (x, bnc, w, b)]
    out = group_norm_act_f(xg[0], G, xg[2], xg[3], 1e-6, act, xg[1])
    out.backward(dy.to(hip))
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), rtol=0, atol=2e-5)
    for a, r, tol in zip(xg, xs, (5e-5, 2e-3, 2e-3, 2e-3)):
        np.testing.assert_allclose(a.grad.cpu().numpy(), r.grad.numpy(), rtol=1e-4,
                                   atol=tol * max(1.0, r.grad.abs().max().item()))


def test_residual_rescale(hip):
    from op.norm_act import residual_rescale
    x, h = torch.randn(2, 6, 5, 7), torch.randn(2, 6, 5, 7)
    b = torch.randn(6)
    out = residual_rescale(x.to(hip), h.to(hip), b.to(hip), np.sqrt(2.)).cpu()
    assert torch.equal(out, (x + (h + b[None, :, None, None])) / np.sqrt(2.))


# ------------------------------------------------------------------ ns_step
def _ns_fields(B, nx, ny, seed=0):
    rng = np.random.default_rng(seed)
    f = rng.uniform(0.1, 1.0, (B, 1, nx, ny)).astype(np.float32)
    p = rng.normal(0, 0.01, (B, 1, nx, ny)).astype(np.float32)
    v = (rng.uniform(0.05, 0.5, (B, 2, nx, ny)) * rng.choice([-1, 1], (B, 2, nx, ny))).astype(np.float32)
    return f, v, p


@pytest.mark.parametrize("B,nx,ny", [(1, 16, 16), (3, 32, 32), (4, 24, 40), (1100, 8, 8),
                                      (2, 192, 192)])
@pytest.mark.parametrize("compat", [True, False])
def test_ns_step_bit_exact_vs_c_oracle(hip, B, nx, ny, compat):
    from op import ns_step
    dt, dx = 0.0025, 0.005
    f, v, p = _ns_fields(B, nx, ny)
    ft, vt, pt = (torch.tensor(a, device=hip) for a in (f, v, p))
    v1 = ns_step.update_velocity(vt, pt, dt, dx, compat=compat).cpu().numpy()
    np.testing.assert_array_equal(v1, ns_step_ref.update_velocity(v, p, dt, dx, compat))
    p1 = ns_step.update_pressure(pt, vt, dt, dx).cpu().numpy()
    np.testing.assert_array_equal(p1, ns_step_ref.update_pressure(p, v, dt, dx))
    f1 = ns_step.update_density(ft, vt, dt, dx).cpu().numpy()
    np.testing.assert_array_equal(f1, ns_step_ref.update_density(f, v, dt, dx))
    # fused whole step == the three reference calls, bit for bit
    d2, v2, p2 = (t.cpu().numpy() for t in ns_step.full_step(ft, vt, pt, dt, dx, compat=compat))
    rd, rv, rp = ns_step_ref.full_step(f, v, p, dt, dx, compat)
    np.testing.assert_array_equal(v2, rv)
    np.testing.assert_array_equal(p2, rp)
    np.testing.assert_array_equal(d2, rd)


@pytest.mark.parametrize("dt,dx", [(0.0037, 0.013), (0.5, 0.9), (1e-4, 2e-3)])
def test_ns_step_bit_exact_varied_steps_and_degenerate_values(hip, dt, dx):
    """Other (dt, dx) pairs, quantised fields (many exactly equal neighbours -> zero
    differences), exact-zero velocities (the reference's division-by-zero NaNs) and a
    wide magnitude range: the fast exactly-rounded divisions must still match."""
    from op import ns_step
    rng = np.random.default_rng(3)
    B, nx, ny = 3, 40, 24
    f = np.round(rng.uniform(0, 4, (B, 1, nx, ny))).astype(np.float32) * 0.25
    p = (rng.normal(0, 1, (B, 1, nx, ny)) * 10.0 ** rng.integers(-6, 3, (B, 1, nx, ny)))
    p = p.astype(np.float32)
    v = rng.uniform(-0.5, 0.5, (B, 2, nx, ny)).astype(np.float32)
    v[rng.random(v.shape) < 0.05] = 0.0
    ft, vt, pt = (torch.tensor(a, device=hip) for a in (f, v, p))
    for compat in (True, False):
        d2, v2, p2 = (t.cpu().numpy() for t in ns_step.full_step(ft, vt, pt, dt, dx, compat=compat))
        rd, rv, rp = ns_step_ref.full_step(f, v, p, dt, dx, compat)
        np.testing.assert_array_equal(v2, rv)
        np.testing.assert_array_equal(p2, rp)
        np.testing.assert_array_equal(d2, rd)
        v1 = ns_step.update_velocity(vt, pt, dt, dx, compat=compat).cpu().numpy()
        np.testing.assert_array_equal(v1, ns_step_ref.update_velocity(v, p, dt, dx, compat))
    np.testing.assert_array_equal(ns_step.update_density(ft, vt, dt, dx).cpu().numpy(),
                                  ns_step_ref.update_density(f, v, dt, dx))


def test_ns_step_nan_quirk_on_zero_velocity(hip):
    from op import ns_step
    f = torch.rand(1, 1, 8, 8, device=hip)
    assert torch.isnan(ns_step.update_density(f, torch.zeros(1, 2, 8, 8, device=hip), 0.1, 0.1)).any()


# ------------------------------------------------------------------ grid_sample
@pytest.mark.parametrize("pm", ["zeros", "border"])
@pytest.mark.parametrize("ac", [True, False])
def test_grid_sample_fwd_bwd_vs_aten_cpu(hip, pm, ac):
    from op.grid_sample import grid_sample_2d
    torch.manual_seed(1)
    inp = torch.randn(3, 5, 9, 11)
    grid = torch.rand(3, 7, 6, 2) * 2.4 - 1.2
    gout = torch.randn(3, 5, 7, 6)
    ri, rg = inp.clone().requires_grad_(True), grid.clone().requires_grad_(True)
    ref = F.grid_sample(ri, rg, mode="bilinear", padding_mode=pm, align_corners=ac)
    ref.backward(gout)
    gi, gg = inp.to(hip).requires_grad_(True), grid.to(hip).requires_grad_(True)
    out = grid_sample_2d(gi, gg, pm, ac)
    out.backward(gout.to(hip))
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), atol=1e-5)
    np.testing.assert_allclose(gi.grad.cpu().numpy(), ri.grad.numpy(), atol=1e-5)
    np.testing.assert_allclose(gg.grad.cpu().numpy(), rg.grad.numpy(), atol=1e-4)


@pytest.mark.parametrize("pm", [0, 1])
def test_grid_sample_grad2_vs_oracle(hip, pm):
    from op.grid_sample import grid_sample2d_grad2_raw
    torch.manual_seed(2)
    N, C, H, W, Ho, Wo = 2, 4, 7, 8, 5, 6
    inp = torch.randn(N, C, H, W, dtype=torch.float64)
    grid = torch.rand(N, Ho, Wo, 2, dtype=torch.float64) * 2.4 - 1.2
    gout = torch.randn(N, C, Ho, Wo, dtype=torch.float64)
    g2i, g2g = torch.randn_like(inp), torch.randn_like(grid)
    ref = grid_sample_ref.grad2(g2i, g2g, gout, inp, grid, pm, True)
    got = grid_sample2d_grad2_raw(*(t.to(hip) for t in (g2i, g2g, gout, inp, grid)), pm, True)
    for a, r in zip(got, ref):
        np.testing.assert_allclose(a.cpu().numpy(), r.numpy(), rtol=1e-10, atol=1e-10)


def test_grid_sample_double_backward_gradgradcheck(hip):
    """Second derivatives through grid_sample, as the PINN residual needs (pinn.py:89-92)."""
    from op.grid_sample import grid_sample_2d
    torch.manual_seed(3)
    inp = torch.randn(1, 2, 5, 5, dtype=torch.float64, device=hip, requires_grad=True)
    grid = (torch.rand(1, 3, 4, 2, dtype=torch.float64, device=hip) * 1.6 - 0.8).requires_grad_(True)
    f = lambda a, g: grid_sample_2d(a, g, "border", True)
    assert torch.autograd.gradcheck(f, (inp, grid))
    assert torch.autograd.gradgradcheck(f, (inp, grid))


def test_grid_sample_double_backward_noncontiguous_views(hip):
    """As flownet.project calls it: the grid an NHWC permute of an NCHW flow, the input a
    channel slice -- both non-contiguous.  A dense copy made inside the Function and saved
    would cut the double backward's grad_grid / grad_input from the graph (caught by the
    float64-truth PINN fixtures); gradgradcheck through the views pins that it flows."""
    from op.grid_sample import grid_sample_2d
    torch.manual_seed(4)
    base = torch.randn(2, 4, 5, 6, dtype=torch.float64, device=hip, requires_grad=True)
    flow = (torch.rand(2, 2, 3, 4, dtype=torch.float64, device=hip) * 1.6 - 0.8).requires_grad_(True)

    def f(b, fl):
        inp = b[:, 1:3]                  # channel slice: non-contiguous
        g = (fl * 0.9).permute(0, 2, 3, 1)  # NHWC view of NCHW
        assert not inp.is_contiguous() and not g.is_contiguous()
        return grid_sample_2d(inp, g, "border", True)

    assert torch.autograd.gradcheck(f, (base, flow))
    assert torch.autograd.gradgradcheck(f, (base, flow))


# ------------------------------------------------------------------ Winograd conv3x3
@pytest.mark.parametrize("N,cin,cout,hw", [(1, 8, 128, 16), (3, 24, 128, 32), (2, 128, 256, 64),
                                           (2, 256, 128, 16), (1, 512, 256, 32),
                                           (9, 64, 128, 64), (16, 16, 64, 96),
                                           (2, 16, 16, 64), (3, 32, 32, 32), (2, 64, 96, 16),
                                           (1, 96, 192, 32)])
@pytest.mark.parametrize("with_bias", [True, False])
def test_conv3x3_winograd_matches_fp32_reference(hip, N, cin, cout, hw, with_bias):
    """Fused Winograd F(2x2,3x3) MFMA conv vs a float64 direct convolution; the fp32 MIOpen
    result is held to the same bound.  Tolerance 2e-5 relative to max|ref| (Winograd's
    transforms add a few rounding steps per term; the network-level tolerance is 1e-4)."""
    import torch.nn.functional as F
    from op.conv import conv3x3
    g = torch.Generator().manual_seed(N * 1000 + cin)
    x = torch.randn(N, cin, hw, hw, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    b = torch.randn(cout, generator=g) if with_bias else None
    ref = F.conv2d(x.double(), w.double(), None if b is None else b.double(), padding=1)
    out = conv3x3(x.to(hip), w.to(hip), None if b is None else b.to(hip)).double().cpu()
    scale = ref.abs().max().item()
    assert (out - ref).abs().max().item() <= 2e-5 * scale
    mi = F.conv2d(x.to(hip), w.to(hip), None if b is None else b.to(hip), padding=1).double().cpu()
    assert (mi - ref).abs().max().item() <= 2e-5 * scale


@pytest.mark.parametrize("cin", [16, 64])
def test_conv3x3_winograd_backward_and_filter_cache(hip, cin):
    """gradients vs MIOpen's; cin = 64 takes the Winograd backward-data path (the forward
    conv of gy with the flipped, transposed filter), cin = 16 the MIOpen fallback."""
    import torch.nn.functional as F
    from op.conv import conv3x3
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, cin, 16, 32, generator=g).to(hip).requires_grad_()
    w = (torch.randn(128, cin, 3, 3, generator=g) * 0.1).to(hip).requires_grad_()
    b = torch.randn(128, generator=g).to(hip).requires_grad_()
    go = torch.randn(2, 128, 16, 32, generator=g).to(hip)
    gx, gw, gb = torch.autograd.grad(conv3x3(x, w, b), (x, w, b), go)
    rx, rw, rb = torch.autograd.grad(F.conv2d(x, w, b, padding=1), (x, w, b), go)
    for a, r in ((gx, rx), (gw, rw), (gb, rb)):
        assert (a - r).abs().max().item() <= 3e-5 * r.abs().max().item()
    # an in-place weight update invalidates the cached filter transform
    y0 = conv3x3(x.detach(), w.detach(), None)
    with torch.no_grad():
        w.mul_(2.0)
    y1 = conv3x3(x.detach(), w.detach(), None)
    assert torch.allclose(y1, 2 * y0, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("N,cin,cout,h,w", [(1, 32, 64, 2, 16), (2, 64, 128, 16, 32),
                                             (3, 96, 64, 10, 48), (2, 256, 128, 32, 32),
                                             (1, 32, 128, 2, 16), (4, 128, 256, 64, 64),
                                             (3, 64, 384, 18, 16), (128, 256, 256, 8, 8),
                                             (2, 32, 64, 8, 8), (16, 512, 256, 8, 8),
                                             (4, 128, 16, 64, 64), (2, 64, 32, 32, 32),
                                             (3, 192, 96, 32, 32), (2, 64, 160, 16, 16),
                                             (4, 32, 48, 8, 8)])
def test_conv3x3_winograd_weight_gradient(hip, N, cin, cout, h, w):
    """Winograd split-K weight gradient vs a float64 direct computation (and MIOpen's fp32
    backward-weights held to the same bound): 2e-5 relative to max|ref|.  Shapes cover one
    K-chunk, several chunks per split, odd strip counts, the NCSN++ channel widths, and the
    pair form for 8-pixel-wide images (two images per strip: CIFAR-10's 8 x 8 level)."""
    import torch.nn.functional as F
    from op import conv as conv_mod
    from op.conv import conv3x3_wgrad_raw
    g = torch.Generator().manual_seed(N * 100 + cin + h)
    x = torch.randn(N, cin, h, w, generator=g)
    gy = torch.randn(N, cout, h, w, generator=g)
    wt = torch.empty(cout, cin, 3, 3)
    assert conv_mod.lib.bpk_conv3x3_wino_wgrad_supported(N, cin, cout, h, w)
    ref = torch.nn.grad.conv2d_weight(x.double(), wt.shape, gy.double(), padding=1)
    out = conv3x3_wgrad_raw(x.to(hip), gy.to(hip), wt.shape).double().cpu()
    scale = ref.abs().max().item()
    assert (out - ref).abs().max().item() <= 2e-5 * scale
    mi = torch.nn.grad.conv2d_weight(x.to(hip), wt.shape, gy.to(hip), padding=1).double().cpu()
    assert (mi - ref).abs().max().item() <= 2e-5 * scale
    # deterministic: the same inputs give the same bits
    again = conv3x3_wgrad_raw(x.to(hip), gy.to(hip), wt.shape).double().cpu()
    assert torch.equal(out, again)
    # the bias gradient from the same kernel: dw unchanged, db = sum of gy over (n, h, w)
    dw2, db = conv3x3_wgrad_raw(x.to(hip), gy.to(hip), wt.shape, bias_grad=True)
    assert torch.equal(dw2.double().cpu(), out)
    dref = gy.double().sum((0, 2, 3))
    assert (db.double().cpu() - dref).abs().max().item() <= 1e-5 * max(1.0, dref.abs().max().item())
    del F


def test_conv3x3_winograd_fused_residual_tail(hip):
    """conv3x3(h, w, b, skip=x, div) == residual_rescale(x, conv3x3(h, w), b, div) bit for bit
    (same epilogue arithmetic), and its gradients match the unfused composition."""
    from op.conv import conv3x3
    from op.norm_act import residual_rescale
    g = torch.Generator().manual_seed(3)
    h = torch.randn(2, 64, 16, 32, generator=g).to(hip).requires_grad_()
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.05).to(hip).requires_grad_()
    b = torch.randn(64, generator=g).to(hip).requires_grad_()
    x = torch.randn(2, 64, 16, 32, generator=g).to(hip).requires_grad_()
    div = float(np.sqrt(2.0))
    fused = conv3x3(h, w, b, skip=x, div=div)
    plain = residual_rescale(x, conv3x3(h, w), b, div)
    assert torch.equal(fused, plain)
    go = torch.randn_like(fused)
    g1 = torch.autograd.grad(fused, (h, w, b, x), go)
    g2 = torch.autograd.grad(plain, (h, w, b, x), go)
    for a, r in zip(g1, g2):
        assert (a - r).abs().max().item() <= 1e-5 * max(1.0, r.abs().max().item())


def test_conv3x3_winograd_fused_groupnorm_silu_prologue(hip):
    """conv3x3(x, pre=group_norm_affine(x, gn, b)) == conv3x3(SiLU(GroupNorm(x + b))) up to
    fp32 rounding of the folded affine form (1e-5 relative), incl. the residual tail."""
    from op.conv import conv3x3
    from op.norm_act import ACT_SILU, group_norm_act, group_norm_affine
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(2, 128, 32, 32, generator=g) * 3 + 1).to(hip)
    gn = torch.nn.GroupNorm(32, 128, eps=1e-6).to(hip)
    with torch.no_grad():
        gn.weight.copy_(torch.rand(128, generator=g) + 0.5)
        gn.bias.copy_(torch.randn(128, generator=g))
        bnc = torch.randn(2, 128, generator=g).to(hip)
        w = (torch.randn(64, 128, 3, 3, generator=g) * 0.03).to(hip)
        b = torch.randn(64, generator=g).to(hip)
        skip = torch.randn(2, 64, 32, 32, generator=g).to(hip)
        ref = conv3x3(group_norm_act(x, gn, ACT_SILU, bnc), w, b, skip=skip, div=2 ** 0.5)
        out = conv3x3(x, w, b, skip=skip, div=2 ** 0.5, pre=group_norm_affine(x, gn, bnc))
    assert (out - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


@pytest.mark.parametrize("cin,cout,hw,two", [(128, 128, 32, False), (256, 256, 16, False),
                                             (384, 128, 32, True), (64, 192, 16, False)])
def test_conv3x3_winograd_prologue_8wave_form(hip, cin, cout, hw, two):
    """The GroupNorm+SiLU prologue conv without a residual tail runs on the 8-wave, 128-cout
    workgroup form when Cout % 128 == 0 (csrc/conv_winograd.hip wino_f23_pipe_kernel<1, true,
    8>; Cout = 192 pads to 256): output and GroupNorm partial statistics vs SiLU(GroupNorm(x))
    through the plain 4-wave kernel and vs F.conv2d in fp32 (1e-5 relative), incl. the up
    path's two-source form."""
    import torch.nn.functional as F
    from op.conv import conv3x3, conv3x3_fwd_raw, gn_partials
    from op.norm_act import ACT_SILU, group_norm_act, group_norm_affine
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(3, cin, hw, hw, generator=g) * 2 + 0.5).to(hip)
    gn = torch.nn.GroupNorm(32, cin, eps=1e-6).to(hip)
    with torch.no_grad():
        gn.weight.copy_(torch.rand(cin, generator=g) + 0.5)
        gn.bias.copy_(torch.randn(cin, generator=g))
        w = (torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)).to(hip)
        b = torch.randn(cout, generator=g).to(hip)
        a = group_norm_act(x, gn, ACT_SILU)
        ref = F.conv2d(a, w, b, padding=1)
        plain = conv3x3(a, w, b)
        pre = group_norm_affine(x, gn)
        if two:
            c1 = cin // 3
            out = conv3x3_fwd_raw(x[:, :c1].contiguous(), w, b, pre=pre, stats=True,
                                  x2=x[:, c1:].contiguous())
        else:
            out = conv3x3(x, w, b, pre=pre, stats=True)
    scale = ref.abs().max().item()
    assert (out - ref).abs().max().item() <= 1e-5 * scale
    assert (out - plain).abs().max().item() <= 1e-5 * scale
    part, R, cnt = gn_partials(out)
    assert R == (hw // 8) * (hw // 16) and cnt == 128
    m = out.reshape(3, cout, hw // 8, 8, hw // 16, 16).mean((3, 5)).reshape(3, cout, R)
    assert (part[..., 0] - m).abs().max().item() <= 1e-5 * scale


# ------------------------------------------------------------------ small-channel conv3x3
@pytest.mark.parametrize("N,cin,cout,h,w", [(2, 1, 128, 128, 128), (3, 3, 64, 20, 36),
                                             (2, 128, 1, 64, 64), (2, 256, 1, 16, 16),
                                             (1, 37, 3, 18, 68), (2, 2, 4, 8, 12),
                                             (1, 4, 2, 33, 100)])
@pytest.mark.parametrize("with_bias", [True, False])
def test_conv3x3_small_channel_matches_fp32_reference(hip, N, cin, cout, h, w, with_bias):
    """Small-channel VALU conv (Cin <= 4 or Cout <= 4: NCSN++ conv_in and pyramid heads) vs a
    float64 direct convolution, 2e-6 relative to max|ref| (plain fp32 FMA chains); shapes
    cover partial 16 x 64 tiles, both kernel forms and ragged channel chunks."""
    from op.conv import conv3x3, small_supported
    g = torch.Generator().manual_seed(N * 7 + cin * 3 + cout)
    x = torch.randn(N, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    b = torch.randn(cout, generator=g) if with_bias else None
    assert small_supported(x.to(hip), wt.to(hip))
    ref = F.conv2d(x.double(), wt.double(), None if b is None else b.double(), padding=1)
    out = conv3x3(x.to(hip), wt.to(hip), None if b is None else b.to(hip)).double().cpu()
    assert (out - ref).abs().max().item() <= 2e-6 * ref.abs().max().item()


@pytest.mark.parametrize("cin,cout", [(1, 64), (64, 1), (3, 2)])
def test_conv3x3_small_channel_backward(hip, cin, cout):
    """input / weight / bias gradients of the small-channel conv vs MIOpen (the input
    gradient runs on the other small-channel form with the flipped, transposed filter)."""
    from op.conv import conv3x3
    g = torch.Generator().manual_seed(cin + 10 * cout)
    x = torch.randn(2, cin, 24, 40, generator=g).to(hip).requires_grad_()
    w = (torch.randn(cout, cin, 3, 3, generator=g) * 0.2).to(hip).requires_grad_()
    b = torch.randn(cout, generator=g).to(hip).requires_grad_()
    go = torch.randn(2, cout, 24, 40, generator=g).to(hip)
    got = torch.autograd.grad(conv3x3(x, w, b), (x, w, b), go)
    ref = torch.autograd.grad(F.conv2d(x, w, b, padding=1), (x, w, b), go)
    for a, r in zip(got, ref):
        assert (a - r).abs().max().item() <= 2e-5 * r.abs().max().item()


def test_conv3x3_small_channel_groupnorm_prologue_and_skip(hip):
    """pyramid head form: conv(SiLU(GroupNorm(x)), Cout = 1) with the normalization applied in
    the kernel's patch load == the unfused composition (1e-5 relative); skip + div tail."""
    from op.conv import conv3x3
    from op.norm_act import ACT_SILU, group_norm_act, group_norm_affine
    g = torch.Generator().manual_seed(9)
    x = (torch.randn(2, 128, 32, 32, generator=g) * 2 + 0.5).to(hip)
    gn = torch.nn.GroupNorm(32, 128, eps=1e-6).to(hip)
    with torch.no_grad():
        gn.weight.copy_(torch.rand(128, generator=g) + 0.5)
        gn.bias.copy_(torch.randn(128, generator=g))
        w = (torch.randn(1, 128, 3, 3, generator=g) * 0.03).to(hip)
        b = torch.randn(1, generator=g).to(hip)
        skip = torch.randn(2, 1, 32, 32, generator=g).to(hip)
        ref = F.conv2d(group_norm_act(x, gn, ACT_SILU), w, b, padding=1)
        out = conv3x3(x, w, b, pre=group_norm_affine(x, gn))
        assert (out - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
        tail = conv3x3(x, w, b, skip=skip, div=2.0, pre=group_norm_affine(x, gn))
        assert (tail - (skip + ref) / 2.0).abs().max().item() <= 1e-5 * ref.abs().max().item()


def test_conv3x3_winograd_many_items_odd_batch(hip):
    """More work items than resident workgroups on an odd batch and non-power-of-two plane
    (11 x 6 x 5 regions, the XCD remap off): GroupNorm prologue + residual tail vs the
    unfused composition in float64 (1e-5 relative)."""
    from op.conv import conv3x3
    from op.norm_act import group_norm_affine
    g = torch.Generator().manual_seed(11)
    N, C, Co, H, W = 11, 64, 128, 48, 80   # 11 * 6 * 5 * 2 = 660 items
    x = (torch.randn(N, C, H, W, generator=g) * 2 + 0.3)
    gn = torch.nn.GroupNorm(16, C, eps=1e-6)
    with torch.no_grad():
        gn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        gn.bias.copy_(torch.randn(C, generator=g))
    w = torch.randn(Co, C, 3, 3, generator=g) * 0.05
    b = torch.randn(Co, generator=g)
    skip = torch.randn(N, Co, H, W, generator=g)
    a = F.silu(F.group_norm(x.double(), 16, gn.weight.double(), gn.bias.double(), 1e-6))
    ref = (skip.double() + F.conv2d(a, w.double(), b.double(), padding=1)) / 2 ** 0.5
    gnd = gn.to(hip)
    with torch.no_grad():
        xd = x.to(hip)
        out = conv3x3(xd, w.to(hip), b.to(hip), skip=skip.to(hip), div=2 ** 0.5,
                      pre=group_norm_affine(xd, gnd)).double().cpu()
    assert (out - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


@pytest.mark.parametrize("with_bias_nc", [False, True])
def test_conv3x3_winograd_gn_partial_statistics(hip, with_bias_nc):
    """GroupNorm partial statistics from the Winograd epilogue (stats=True, incl. the residual
    tail) and through a channel concat: the affine form built from them equals the one from
    the full statistics pass (1e-5 relative), and the conv output itself is unchanged."""
    from models.layers import cat_channels
    from op.conv import conv3x3, gn_partials
    from op.norm_act import group_norm_affine
    g = torch.Generator().manual_seed(21)
    N, C, Co, H, W = 3, 64, 128, 32, 48
    x = torch.randn(N, C, H, W, generator=g).to(hip)
    w = (torch.randn(Co, C, 3, 3, generator=g) * 0.05).to(hip)
    b = torch.randn(Co, generator=g).to(hip)
    skip = (torch.randn(N, Co, H, W, generator=g) * 3 + 1).to(hip)
    other = (torch.randn(N, Co, H, W, generator=g) * 0.5 - 2).to(hip)
    bnc = torch.randn(N, 2 * Co, generator=g).to(hip) if with_bias_nc else None
    gn = torch.nn.GroupNorm(32, 2 * Co, eps=1e-6).to(hip)
    with torch.no_grad():
        gn.weight.copy_((torch.rand(2 * Co, generator=g) + 0.5).to(hip))
        gn.bias.copy_(torch.randn(2 * Co, generator=g).to(hip))
        y = conv3x3(x, w, b, skip=skip, div=2 ** 0.5, stats=True)
        y2 = conv3x3(skip, w.new_zeros(Co, Co, 3, 3) + 0.01, None, skip=other, div=1.0, stats=True)
        assert gn_partials(y) is not None and gn_partials(y2) is not None
        plain = conv3x3(x, w, b, skip=skip, div=2 ** 0.5)
        assert torch.equal(y, plain)
        cat = cat_channels(y, y2)
        assert gn_partials(cat) is not None
        got = group_norm_affine(cat, gn, bnc)
        ref = group_norm_affine(cat.clone(), gn, bnc)   # clone: no partials -> full pass
        assert (got - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
        # the two parts' partials read in place == the concatenated partials (bit-identical),
        # also when a group straddles the boundary (192 channels / 32 groups, C1 = 128)
        from op.norm_act import group_norm_affine_partials
        two = group_norm_affine_partials(gn_partials(y), N, 2 * Co, gn, bnc, part2=gn_partials(y2))
        assert torch.equal(two, got)
        y3 = conv3x3(skip, w.new_zeros(64, Co, 3, 3) + 0.02, None, stats=True)
        gn3 = torch.nn.GroupNorm(32, Co + 64, eps=1e-6).to(hip)
        cat3 = cat_channels(y, y3)
        two3 = group_norm_affine_partials(gn_partials(y), N, Co + 64, gn3, None,
                                          part2=gn_partials(y3))
        assert torch.equal(two3, group_norm_affine(cat3, gn3))
        ref3 = group_norm_affine(cat3.clone(), gn3)
        assert (two3 - ref3).abs().max().item() <= 1e-5 * ref3.abs().max().item()
        # partials computed from a plain tensor (one pass) give the same affine form
        from op.conv import ensure_gn_partials
        plain2 = cat.clone()
        assert gn_partials(plain2) is None and ensure_gn_partials(plain2) is not None
        got2 = group_norm_affine(plain2, gn, bnc)
        assert (got2 - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
        # an in-place update invalidates the attached statistics
        y.add_(1.0)
        assert gn_partials(y) is None


@pytest.mark.parametrize("cin,cout", [(32, 2), (4, 64)])
def test_conv3x3_small_channel_double_backward(hip, cin, cout):
    """Second derivatives through the small-channel conv (the PINN residual differentiates
    the networks twice): grad of <d out/d x . v> w.r.t. x and w vs MIOpen's (2e-5 relative)."""
    from op.conv import conv3x3
    g = torch.Generator().manual_seed(cin * 7 + cout)
    x0 = torch.randn(2, cin, 16, 24, generator=g)
    w0 = torch.randn(cout, cin, 3, 3, generator=g) * 0.2
    go = torch.randn(2, cout, 16, 24, generator=g).to(hip)
    v = torch.randn(2, cin, 16, 24, generator=g).to(hip)

    def second(fn):
        x = x0.to(hip).requires_grad_()
        w = w0.to(hip).requires_grad_()
        y = fn(x, w)
        (gx,) = torch.autograd.grad(y, x, go, create_graph=True)
        return torch.autograd.grad((gx * v).sum() + (gx * gx).sum(), (x, w))

    got = second(lambda x, w: conv3x3(torch.tanh(x), w))
    ref = second(lambda x, w: F.conv2d(torch.tanh(x), w, padding=1))
    for a, r in zip(got, ref):
        assert (a - r).abs().max().item() <= 2e-5 * max(1e-6, r.abs().max().item())


@pytest.mark.parametrize("cin,cout,hw", [(64, 128, (16, 32)), (16, 32, (12, 20)), (64, 32, (16, 16))])
def test_conv3x3_double_backward_any_shape(hip, cin, cout, hw):
    """Second derivatives through conv3x3 for Winograd-eligible (64 -> 128) and MIOpen-fallback
    shapes: the backward is expressed in conv3x3 / weight-gradient ops that are themselves
    differentiable; grads of a function of (dL/dx, dL/dw) w.r.t. x and w vs F.conv2d's
    (2e-5 relative)."""
    from op.conv import conv3x3
    g = torch.Generator().manual_seed(cin + cout)
    x0 = torch.randn(2, cin, *hw, generator=g)
    w0 = torch.randn(cout, cin, 3, 3, generator=g) * 0.1
    b0 = torch.randn(cout, generator=g)
    go = torch.randn(2, cout, *hw, generator=g).to(hip)
    v = torch.randn(2, cin, *hw, generator=g).to(hip)

    def second(fn):
        x = x0.to(hip).requires_grad_()
        w = w0.to(hip).requires_grad_()
        b = b0.to(hip).requires_grad_()
        y = fn(torch.tanh(x), w, b)
        gx, gw = torch.autograd.grad(y, (x, w), go, create_graph=True)
        return torch.autograd.grad((gx * v).sum() + (gw * gw).sum() + (gx * gx).sum(), (x, w, b),
                                   allow_unused=True)

    got = second(lambda x, w, b: conv3x3(x, w, b))
    ref = second(lambda x, w, b: F.conv2d(x, w, b, padding=1))
    for a, r in zip(got, ref):
        if r is None:
            assert a is None or a.abs().max().item() == 0
            continue
        assert (a - r).abs().max().item() <= 2e-5 * max(1e-6, r.abs().max().item())


@pytest.mark.parametrize("N,k1,k2,m,hw", [(2, 64, 0, 128, 16), (3, 128, 64, 256, 32),
                                          (1, 256, 256, 128, 16), (2, 16, 48, 384, 32),
                                          (2, 96, 0, 32, 16), (1, 64, 32, 80, 16),
                                          (8, 256, 0, 256, 16), (8, 512, 0, 768, 16),
                                          (4, 128, 128, 144, 16), (8, 256, 256, 256, 32)])
def test_conv1x1_gemm_matches_fp32_reference(hip, N, k1, k2, m, hw):
    """MFMA 1x1-conv GEMM (one or two sources along K) vs float64 (1e-5 relative); the
    two-source form equals conv1x1 of the concatenation.  The small-batch cases take the
    split-K form (bpk_gemm_nchw_splitk_f32: the 16^2 / 32^2 levels at 8 samples per GPU),
    incl. a split that crosses the two sources and an M that is not a multiple of 128."""
    from op.conv import conv1x1, lib
    if N >= 4:
        assert lib.bpk_gemm_nchw_splitk_bytes(N, m, hw * hw, k1, k2) > 0
    g = torch.Generator().manual_seed(k1 + k2 + m)
    x1 = torch.randn(N, k1, hw, hw, generator=g)
    x2 = torch.randn(N, k2, hw, hw, generator=g) if k2 else None
    w = torch.randn(m, k1 + k2, 1, 1, generator=g) / (k1 + k2) ** 0.5
    b = torch.randn(m, generator=g)
    xc = x1 if x2 is None else torch.cat([x1, x2], 1)
    ref = F.conv2d(xc.double(), w.double(), b.double())
    with torch.no_grad():
        out = conv1x1(x1.to(hip), w.to(hip), b.to(hip), None if x2 is None else x2.to(hip))
    assert (out.double().cpu() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


@pytest.mark.parametrize("N,k,m,hw", [(1, 128, 128, 4), (2, 128, 256, 16), (3, 384, 128, 20),
                                     (8, 256, 256, 64), (2, 64, 16, 16), (3, 96, 192, 8),
                                     (2, 448, 96, 32)])
def test_conv1x1_wgrad_gemm_matches_fp64(hip, N, k, m, hw):
    """1x1 weight / bias gradient GEMM (split-K over pixels, one split and many) vs float64:
    dw = sum_n gy[n] x[n]^T, db = gy.sum((0, 2, 3)) (1e-5 relative); deterministic."""
    from op.conv import _wgrad1x1_raw
    g = torch.Generator().manual_seed(N * 1000 + k + m + hw)
    x = torch.randn(N, k, hw, hw, generator=g)
    gy = torch.randn(N, m, hw, hw, generator=g)
    ref_w = torch.einsum("nmp,nkp->mk", gy.double().flatten(2), x.double().flatten(2))
    ref_b = gy.double().sum((0, 2, 3))
    dw, db = _wgrad1x1_raw(gy.to(hip), x.to(hip), True)
    assert (dw.double().cpu() - ref_w).abs().max().item() <= 1e-5 * ref_w.abs().max().item()
    assert (db.double().cpu() - ref_b).abs().max().item() <= 1e-5 * ref_b.abs().max().item()
    dw2, _ = _wgrad1x1_raw(gy.to(hip), x.to(hip), False)
    assert torch.equal(dw, dw2)


@pytest.mark.parametrize("cin,cout,hw", [(128, 256, 16), (256, 128, 32), (384, 128, 16),
                                         (64, 16, 16), (96, 192, 16), (448, 96, 32)])
def test_conv1x1_autograd_double_backward(hip, cin, cout, hw):
    """conv1x1_ad (GEMM kernels for the forward, its adjoint and the weight / bias gradient,
    each differentiable again) vs F.conv2d: forward, first and second derivatives w.r.t.
    x, w, b (2e-5 relative)."""
    from op.conv import conv1x1_ad
    g = torch.Generator().manual_seed(cin + cout + hw)
    x0 = torch.randn(2, cin, hw, hw, generator=g)
    w0 = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    b0 = torch.randn(cout, generator=g)
    go = torch.randn(2, cout, hw, hw, generator=g).to(hip)
    v = torch.randn(2, cin, hw, hw, generator=g).to(hip)

    def run(fn):
        x = x0.to(hip).requires_grad_()
        w = w0.to(hip).requires_grad_()
        b = b0.to(hip).requires_grad_()
        y = fn(torch.tanh(x), w, b)
        gx, gw, gb = torch.autograd.grad(y, (x, w, b), go, create_graph=True)
        second = torch.autograd.grad((gx * v).sum() + (gw * gw).sum() + (gx * gx).sum()
                                     + (gb * gb).sum(), (x, w, b), allow_unused=True)
        return (y.detach(), gx.detach(), gw.detach(), gb.detach()) + second

    got = run(conv1x1_ad)
    ref = run(lambda x, w, b: F.conv2d(x, w, b))
    for a, r in zip(got, ref):
        if r is None:
            assert a is None or a.abs().max().item() == 0
            continue
        assert (a - r).abs().max().item() <= 2e-5 * max(1e-6, r.abs().max().item())


def test_conv3x3_winograd_two_sources(hip):
    """The Winograd conv reading [x1, x2] as two sources equals the conv of their
    concatenation (same kernel, same chunk order: bit-identical), incl. the GroupNorm
    prologue and the partial statistics."""
    from op.conv import conv3x3, conv3x3_pair, gn_partials
    g = torch.Generator().manual_seed(31)
    x1 = torch.randn(2, 64, 16, 32, generator=g).to(hip)
    x2 = torch.randn(2, 128, 16, 32, generator=g).to(hip)
    w = (torch.randn(128, 192, 3, 3, generator=g) * 0.03).to(hip)
    b = torch.randn(128, generator=g).to(hip)
    pre = torch.stack([torch.rand(2, 192, generator=g) + 0.5, torch.randn(2, 192, generator=g)], -1).to(hip)
    with torch.no_grad():
        ref = conv3x3(torch.cat([x1, x2], 1), w, b, pre=pre, stats=True)
        out = conv3x3_pair(x1, x2, w, b, pre=pre, stats=True)
    assert torch.equal(out, ref)
    # statistics: same values, merge order may differ between kernel forms
    pa, pb = gn_partials(out)[0], gn_partials(ref)[0]
    assert torch.allclose(pa, pb, rtol=1e-5, atol=1e-6 * pb.abs().max().item())


@pytest.mark.parametrize("hs_stats", [True, False])
def test_resblock_forward_pair_matches_concat(hip, hs_stats):
    """ResnetBlockBigGANpp.forward_pair(h, hs) (no concatenation: partial-statistics
    GroupNorm, two-source Winograd conv, two-source 1x1 GEMM) == forward(cat([h, hs]))
    within 1e-5 relative, and the output carries partial statistics.  hs_stats=False: hs
    comes without partials (they are computed from it in one pass)."""
    import models.layerspp as lpp
    from models.layers import cat_channels
    from op.conv import conv3x3, gn_partials
    torch.manual_seed(0)
    blk = lpp.ResnetBlockBigGANpp(act=torch.nn.SiLU(), in_ch=256, out_ch=128, temb_dim=512,
                                  skip_rescale=True, init_scale=0.).to(hip).eval()
    with torch.no_grad():
        for p in blk.parameters():
            p.add_(torch.randn_like(p) * 0.02)
        g = torch.Generator().manual_seed(4)
        src = torch.randn(2, 64, 32, 32, generator=g).to(hip)
        w1 = (torch.randn(128, 64, 3, 3, generator=g) * 0.05).to(hip)
        w2 = (torch.randn(128, 64, 3, 3, generator=g) * 0.05).to(hip)
        h = conv3x3(src, w1, stats=True)      # producers that attach partial statistics
        hs = conv3x3(src, w2, stats=hs_stats)
        assert gn_partials(h) is not None and (gn_partials(hs) is not None) == hs_stats
        temb = torch.randn(2, 512, generator=g).to(hip)
        out = blk.forward_pair(h, hs, temb)
        ref = blk(cat_channels(h, hs), temb)
    assert (out - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    assert gn_partials(out) is not None


def _count_gn_conv_ad():
    """calls of op.conv._GNSiLUConv3x3.forward from now on"""
    from op import conv
    n = [0]
    orig = conv._GNSiLUConv3x3.forward

    def fwd(ctx, *a):
        n[0] += 1
        return orig(ctx, *a)
    conv._GNSiLUConv3x3.forward = staticmethod(fwd)

    def calls():
        conv._GNSiLUConv3x3.forward = staticmethod(orig)
        return n[0]
    return calls


@pytest.mark.parametrize("kind", ["biggan", "ddpm"])
def test_skip_link_hands_the_skip_gradient_to_the_groupnorm_backward(hip, kind):
    """A residual block with an identity skip in eval mode under autograd (DPS): with the skip
    link (models.layers.skip_link) the second conv's skip gradient is added inside the first
    conv's GroupNorm backward -- d/dx bit-identical to the engine's accumulation (the same fp32
    add), one full-size add launch fewer per block."""
    from torch.utils._python_dispatch import TorchDispatchMode
    import models.layers as layers
    import models.layerspp as lpp
    torch.manual_seed(1)
    if kind == "biggan":
        blk = lpp.ResnetBlockBigGANpp(act=torch.nn.SiLU(), in_ch=128, out_ch=128, temb_dim=64,
                                      skip_rescale=True, init_scale=0., dropout=0.0)
    else:
        blk = layers.ResnetBlockDDPM(act=torch.nn.SiLU(), in_ch=128, out_ch=128, temb_dim=64,
                                     dropout=0.0)
    blk = blk.to(hip).eval()
    g = torch.Generator().manual_seed(7)
    x0 = torch.randn(4, 128, 32, 32, generator=g).to(hip)
    temb = torch.randn(4, 64, generator=g).to(hip)
    gout = torch.randn(4, 128, 32, 32, generator=g).to(hip)

    class Adds(TorchDispatchMode):
        n = 0

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            if func.overloadpacket.__name__ in ("add", "add_"):
                Adds.n += 1
            return func(*args, **(kwargs or {}))

    def dx(link):
        old = layers._SKIP_LINK
        layers._SKIP_LINK = link
        try:
            x = x0.clone().requires_grad_()
            y = blk(x, temb)
            Adds.n = 0
            with Adds():
                (gx,) = torch.autograd.grad(y, x, gout)
            return gx, Adds.n
        finally:
            layers._SKIP_LINK = old
    gl, nl = dx(True)
    gu, nu = dx(False)
    assert torch.equal(gl, gu)
    assert nl == nu - 1, (nl, nu)


@pytest.mark.parametrize("kind,cin,cout,hw", [("biggan", 128, 128, 32), ("biggan", 128, 256, 8),
                                              ("ddpm", 128, 128, 32), ("ddpm", 256, 128, 16)])
def test_gn_silu_conv_under_autograd_matches_unfused(hip, kind, cin, cout, hw):
    """The residual blocks in eval mode under autograd (DPS) with GroupNorm+SiLU inside the
    Winograd convs' input loads (op.conv.gn_silu_conv3x3_ad; 8x8 images on the pair form) ==
    the unfused composition (GroupNorm+SiLU kernel, conv, residual): output, d/dx and every
    parameter gradient (the weight gradient with the prologue in its patch load) within 2e-5
    of the tensor's max; and d/dx alone (the DPS call: torch.autograd.grad w.r.t. the input,
    no weight gradients computed)."""
    import models.layers as layers
    import models.layerspp as lpp
    torch.manual_seed(0)
    if kind == "biggan":
        blk = lpp.ResnetBlockBigGANpp(act=torch.nn.SiLU(), in_ch=cin, out_ch=cout, temb_dim=64,
                                      skip_rescale=True, init_scale=0., dropout=0.0)
    else:
        blk = layers.ResnetBlockDDPM(act=torch.nn.SiLU(), in_ch=cin, out_ch=cout, temb_dim=64,
                                     dropout=0.0)
    blk = blk.to(hip).eval()
    with torch.no_grad():
        for p in blk.parameters():
            p.add_(torch.randn_like(p) * 0.05)
    g = torch.Generator().manual_seed(cin + cout + hw)
    x0 = (torch.randn(4, cin, hw, hw, generator=g) * 1.5 + 0.3).to(hip)
    temb = torch.randn(4, 64, generator=g).to(hip)
    gout = torch.randn(4, cout, hw, hw, generator=g).to(hip)

    def run(fused):
        old = layers._GN_CONV_AD
        layers._GN_CONV_AD = fused
        try:
            blk.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_()
            calls = _count_gn_conv_ad()
            y = blk(x, temb)
            assert (calls() > 0) == fused  # the fused path ran (or did not)
            (y * gout).sum().backward()
            grads = [p.grad.clone() for p in blk.parameters()]
            x2 = x0.clone().requires_grad_()
            gx_only = torch.autograd.grad((blk(x2, temb) * gout).sum(), x2)[0]
        finally:
            layers._GN_CONV_AD = old
        return y.detach(), x.grad, grads, gx_only
    yf, gxf, gpf, gof = run(True)
    yu, gxu, gpu_, gou = run(False)

    def close(a, b, what):
        scale = b.abs().max().item()
        assert (a - b).abs().max().item() <= 2e-5 * scale + 1e-30, what
    close(yf, yu, "output")
    close(gxf, gxu, "d/dx")
    close(gof, gou, "d/dx (input-only call)")
    for (name, _), a, b in zip(blk.named_parameters(), gpf, gpu_):
        close(a, b, name)


@pytest.mark.parametrize("k,stride,pad,cin,cout", [(3, 2, 1, 1, 16), (3, 2, 1, 16, 32), (1, 1, 0, 64, 128)])
def test_conv2d_general_double_backward(hip, k, stride, pad, cin, cout):
    """conv2d_general (MIOpen kernels, derivatives of every order as convolutions / conv
    transposes / weight gradients) vs F.conv2d: forward, and second derivatives w.r.t. x, w, b
    of a function of (dL/dx, dL/dw) (2e-5 relative)."""
    from op.conv import conv2d_general
    g = torch.Generator().manual_seed(k * 100 + stride * 10 + cin)
    x0 = torch.randn(2, cin, 16, 20, generator=g)
    w0 = torch.randn(cout, cin, k, k, generator=g) * 0.2
    b0 = torch.randn(cout, generator=g)
    ho, wo = (16 + 2 * pad - k) // stride + 1, (20 + 2 * pad - k) // stride + 1
    go = torch.randn(2, cout, ho, wo, generator=g).to(hip)
    v = torch.randn(2, cin, 16, 20, generator=g).to(hip)

    def second(fn):
        x = x0.to(hip).requires_grad_()
        w = w0.to(hip).requires_grad_()
        b = b0.to(hip).requires_grad_()
        y = fn(torch.tanh(x), w, b)
        gx, gw = torch.autograd.grad(y, (x, w), go, create_graph=True)
        return (y.detach(),) + torch.autograd.grad(
            (gx * v).sum() + (gw * gw).sum() + (gx * gx).sum(), (x, w, b), allow_unused=True)

    got = second(lambda x, w, b: conv2d_general(x, w, b, stride, pad))
    ref = second(lambda x, w, b: F.conv2d(x, w, b, stride, pad))
    for a, r in zip(got, ref):
        if r is None:
            assert a is None or a.abs().max().item() == 0
            continue
        assert (a - r).abs().max().item() <= 2e-5 * max(1e-6, r.abs().max().item())


@pytest.mark.parametrize("C,hw", [(256, 16), (128, 16)])
def test_attention_qkv_gemm_matches_unfused(hip, C, hw):
    """AttnBlockpp at inference (q, k, v as one GEMM over the stacked NIN weights, scale
    folded into q when 1/sqrt(C) is a power of two) == the per-NIN composition (1e-5 rel)."""
    import models.layerspp as lpp
    from models import layers
    torch.manual_seed(C)
    blk = lpp.AttnBlockpp(channels=C, skip_rescale=True, init_scale=0.).to(hip).eval()
    with torch.no_grad():
        for p in blk.parameters():
            p.add_(torch.randn_like(p) * 0.1)
        x = torch.randn(2, C, hw, hw, device=hip)
        h = layers.gn_act(x, blk.GroupNorm_0, None)
        assert blk._qkv_ok(h)
        got = blk._forward_qkv(h)
        ref = blk.NIN_3(layers._attention(h, blk.NIN_0, blk.NIN_1, blk.NIN_2))
        assert (got - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
        out = blk(x)
        assert (out - lpp.residual_rescale(x, ref, None, 2 ** 0.5)).abs().max().item() <= \
            1e-5 * out.abs().max().item()


@pytest.mark.parametrize("cin,cout", [(32, 16), (16, 32), (64, 96), (32, 192)])
def test_conv3x3_winograd_padded_cout_fused_variants(hip, cin, cout):
    """Cout % 64 != 0 (computed for Cout rounded up to 64, Cout stored): GroupNorm+SiLU
    prologue, residual tail and the output's GroupNorm partial statistics vs the unfused
    torch composition (2e-5 relative); first and second derivatives vs F.conv2d."""
    from op.conv import conv3x3, gn_partials
    from op.norm_act import group_norm_affine
    g = torch.Generator().manual_seed(cin * 31 + cout)
    N, H, W = 2, 16, 32
    x = torch.randn(N, cin, H, W, generator=g).to(hip)
    w = (torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)).to(hip)
    b = torch.randn(cout, generator=g).to(hip)
    skip = torch.randn(N, cout, H, W, generator=g).to(hip)
    pre = torch.stack([torch.rand(N, cin, generator=g) + 0.5,
                       torch.randn(N, cin, generator=g)], -1).to(hip)
    with torch.no_grad():
        a = F.silu(x * pre[..., 0, None, None] + pre[..., 1, None, None])
        ref = (skip + F.conv2d(a, w, b, padding=1)) / 2 ** 0.5
        out = conv3x3(x, w, b, skip=skip, div=2 ** 0.5, pre=pre, stats=True)
        assert (out - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()
        assert gn_partials(out) is not None
        gn = torch.nn.GroupNorm(min(cout // 4, 32), cout, eps=1e-6).to(hip)
        got = group_norm_affine(out, gn)
        full = group_norm_affine(out.clone(), gn)
        assert (got - full).abs().max().item() <= 1e-5 * full.abs().max().item()
    go = torch.randn(N, cout, H, W, generator=g).to(hip)
    v = torch.randn(N, cin, H, W, generator=g).to(hip)

    def second(fn):
        xx = x.clone().requires_grad_()
        ww = w.clone().requires_grad_()
        y = fn(torch.tanh(xx), ww)
        gx, gw = torch.autograd.grad(y, (xx, ww), go, create_graph=True)
        return (gx.detach(), gw.detach()) + torch.autograd.grad(
            (gx * v).sum() + (gw * gw).sum(), (xx, ww))

    got = second(lambda t, ww: conv3x3(t, ww, b))
    refs = second(lambda t, ww: F.conv2d(t, ww, b, padding=1))
    for a_, r_ in zip(got, refs):
        assert (a_ - r_).abs().max().item() <= 2e-5 * max(1e-6, r_.abs().max().item())


@pytest.mark.parametrize("co,ci", [(64, 128), (128, 32), (32, 16), (16, 2)])
def test_conv3x3_backward_data_flip_in_filter_transform(hip, co, ci):
    """conv3x3(dy, flip_t(w)) with the flip / transpose read inside the Winograd filter
    transform (no flipped copy of w; MIOpen / small kernel with an explicit flip where the
    shape does not qualify) == F.conv2d with the flipped weight (2e-5 relative)."""
    from op.conv import _flip_t, _fwd_ft_impl
    g = torch.Generator().manual_seed(co + 7 * ci)
    dy = torch.randn(2, co, 16, 32, generator=g).to(hip)
    w = (torch.randn(co, ci, 3, 3, generator=g) / (3 * co ** 0.5)).to(hip)
    with torch.no_grad():
        got = _fwd_ft_impl(dy, w)
        ref = F.conv2d(dy, _flip_t(w).contiguous(), padding=1)
    assert (got - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()


def test_grad_pruning_input_derivatives_then_parameter_gradients(hip):
    """The PINN pattern: d out / d x with create_graph (the engine runs no parameter edge, so
    the custom Functions skip weight / bias gradients), then a loss of that derivative
    backpropagated to the parameters.  Input derivative and parameter gradients vs the same
    network on F.conv2d (2e-5 relative)."""
    from op.conv import conv3x3, conv1x1_ad
    g = torch.Generator().manual_seed(5)
    x0 = torch.randn(2, 16, 16, 32, generator=g)
    w1 = torch.randn(32, 16, 3, 3, generator=g) * 0.1
    b1 = torch.randn(32, generator=g) * 0.1
    w2 = torch.randn(128, 32, 1, 1, generator=g) * 0.1
    w3 = torch.randn(16, 128, 3, 3, generator=g) * 0.05

    def run(c3, c1):
        ps = [t.to(hip).requires_grad_() for t in (w1, b1, w2, w3)]
        x = x0.to(hip).requires_grad_()
        h = torch.tanh(c3(x, ps[0], ps[1]))
        h = torch.tanh(c1(h, ps[2]))
        y = c3(h, ps[3], None)
        (dx,) = torch.autograd.grad(y.sum(), x, create_graph=True)
        (dx * dx).sum().backward()
        return [dx.detach()] + [p.grad for p in ps]

    got = run(lambda t, w, b: conv3x3(t, w, b), lambda t, w: conv1x1_ad(t, w))
    ref = run(lambda t, w, b: F.conv2d(t, w, b, padding=1), lambda t, w: F.conv2d(t, w))
    for a, r in zip(got, ref):
        assert (a - r).abs().max().item() <= 2e-5 * max(1e-6, r.abs().max().item())


@pytest.mark.parametrize("hw", [(16, 16), (32, 32), (64, 64), (128, 128), (20, 64), (64, 16)])
def test_upfirdn2d_fir_pad2_odd_width_tail_path(hip, hw):
    """FIR-only pad(2, 2) (conv_downsample_2d's FIR, op/upfirdn2d.py:145) on 2^k-wide planes:
    the 2^k + 1 output width takes the streaming kernel's tail-column path; vs the oracle."""
    from op import upfirdn2d
    from oracle.upfirdn2d_ref import upfirdn2d_np
    H, W = hw
    g = torch.Generator().manual_seed(H * 1000 + W)
    x = torch.randn(3, 5, H, W, generator=g)
    k = np.outer([1, 3, 3, 1], [1, 3, 3, 1]).astype(np.float32) / 64
    y = upfirdn2d(x.to(hip), torch.tensor(k, device=hip), pad=(2, 2)).cpu().numpy()
    ref = upfirdn2d_np(x.numpy(), k, (1, 1), (1, 1), (2, 2, 2, 2))
    assert y.shape == ref.shape == (3, 5, H + 1, W + 1)
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-6)


# ------------------------------------------------------------------ grid_sample 3-D
@pytest.mark.parametrize("pm", ["zeros", "border"])
@pytest.mark.parametrize("ac", [True, False])
def test_grid_sample_3d_fwd_bwd_vs_aten_cpu(hip, pm, ac):
    from op.grid_sample import grid_sample_3d
    torch.manual_seed(11)
    inp = torch.randn(2, 3, 5, 6, 7)
    grid = torch.rand(2, 4, 3, 5, 3) * 2.4 - 1.2
    gout = torch.randn(2, 3, 4, 3, 5)
    ri, rg = inp.clone().requires_grad_(True), grid.clone().requires_grad_(True)
    ref = F.grid_sample(ri, rg, mode="bilinear", padding_mode=pm, align_corners=ac)
    ref.backward(gout)
    gi, gg = inp.to(hip).requires_grad_(True), grid.to(hip).requires_grad_(True)
    out = grid_sample_3d(gi, gg, pm, ac)
    out.backward(gout.to(hip))
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), atol=1e-5)
    np.testing.assert_allclose(gi.grad.cpu().numpy(), ri.grad.numpy(), atol=1e-5)
    np.testing.assert_allclose(gg.grad.cpu().numpy(), rg.grad.numpy(), atol=1e-4)


@pytest.mark.parametrize("pm", [0, 1])
def test_grid_sample_3d_grad2_vs_oracle(hip, pm):
    """vs oracle/grid_sample_ref.grad3 (restatement of op/grid_sample_kernel.cu:212-533,
    pinned by finite differences of ATen's first backward, tests/test_grid_sample3d_host.py)"""
    from op.grid_sample import grid_sample3d_grad2_raw
    torch.manual_seed(12)
    d = torch.float64
    inp = torch.randn(2, 3, 4, 5, 6, dtype=d)
    grid = torch.rand(2, 3, 2, 4, 3, dtype=d) * 2.4 - 1.2
    gout = torch.randn(2, 3, 3, 2, 4, dtype=d)
    g2i, g2g = torch.randn_like(inp), torch.randn_like(grid)
    ref = grid_sample_ref.grad3(g2i, g2g, gout, inp, grid, pm, True)
    got = grid_sample3d_grad2_raw(*(t.to(hip) for t in (g2i, g2g, gout, inp, grid)), pm, True)
    for a, r in zip(got, ref):
        np.testing.assert_allclose(a.cpu().numpy(), r.numpy(), rtol=1e-10, atol=1e-10)


def test_grid_sample_3d_double_backward_gradgradcheck(hip):
    from op.grid_sample import grid_sample_3d
    torch.manual_seed(13)
    inp = torch.randn(1, 2, 3, 4, 4, dtype=torch.float64, device=hip, requires_grad=True)
    grid = (torch.rand(1, 2, 3, 2, 3, dtype=torch.float64, device=hip) * 1.6 - 0.8).requires_grad_(True)
    f = lambda a, g: grid_sample_3d(a, g, "border", True)
    assert torch.autograd.gradcheck(f, (inp, grid))
    assert torch.autograd.gradgradcheck(f, (inp, grid))


def test_dispatcher_ops_equal_the_op_wrappers(hip):
    """torch.ops.<reference extension>.* (op/torch_ops.py) run the same kernels as op/*."""
    import op
    from op import ns_step
    from op.grid_sample import grid_sample2d_grad2_raw
    g = torch.Generator().manual_seed(21)
    x = torch.randn(2, 3, 16, 16, generator=g).to(hip)
    k = torch.tensor(np.outer([1, 3, 3, 1], [1, 3, 3, 1]) / 64.0, dtype=torch.float32, device=hip)
    a = torch.ops.upfirdn2d_op.upfirdn2d(x.reshape(6, 16, 16, 1), k, 1, 1, 2, 2, 1, 1, 1, 1)
    assert torch.equal(a.reshape(2, 3, 8, 8), op.upfirdn2d(x, k, down=2, pad=(1, 1)))
    b = torch.randn(3, generator=g).to(hip)
    e = torch.empty(0, device=hip)
    assert torch.equal(torch.ops.fused.fused_bias_act(x, b, e, 3, 0, 0.2, 2 ** 0.5),
                       op.fused_leaky_relu(x, b))
    f = torch.rand(2, 1, 16, 16, generator=g).to(hip) + 0.1
    v = (torch.rand(2, 2, 16, 16, generator=g).to(hip) + 0.05)
    p = torch.randn(2, 1, 16, 16, generator=g).to(hip) * 0.01
    assert torch.equal(torch.ops.ns_step_forward.update_velocity(v, p, 0.0025, 0.005),
                       ns_step.update_velocity(v, p, 0.0025, 0.005))
    inp = torch.randn(2, 3, 5, 6, generator=g, dtype=torch.float64).to(hip)
    grid = (torch.rand(2, 4, 3, 2, generator=g, dtype=torch.float64) * 2 - 1).to(hip)
    go = torch.randn(2, 3, 4, 3, generator=g, dtype=torch.float64).to(hip)
    g2i, g2g = torch.randn_like(inp), torch.randn_like(grid)
    for u, w in zip(torch.ops.gridsample_grad2.grad2_2d(g2i, g2g, go, inp, grid, True, True),
                    grid_sample2d_grad2_raw(g2i, g2g, go, inp, grid, 1, True)):
        assert torch.allclose(u, w, rtol=0, atol=1e-12)


# ------------------------------------------------ implicit-GEMM MFMA conv (conv_igemm.hip)
_IG_CASES = [
    # N, Cin, H, W, Cout, k, stride, pad
    (3, 5, 7, 9, 6, 3, 1, 1),        # odd everything, generic edges
    (2, 16, 16, 20, 32, 3, 2, 1),    # FlowNet pyramid stride-2 conv
    (4, 8, 17, 17, 8, 3, 2, 0),      # FIR conv_downsample_2d (pad 0 after the FIR pad)
    (2, 49, 8, 8, 128, 3, 1, 1),     # FlowNet corr_conv first conv (Cin 49)
    (64, 258, 2, 2, 128, 3, 1, 1),   # refinement conv at 2^2 (split-K)
    (16, 256, 8, 8, 256, 3, 1, 1),   # CIFAR 8^2 level
    (8, 128, 4, 4, 256, 3, 1, 1),    # CIFAR 4^2 level
    (2, 12, 6, 10, 20, 2, 2, 0),     # ConvTranspose2d(k2, s2) adjoint shape
    (2, 6, 9, 9, 4, 4, 2, 1),        # flow_upsample k4 s2 p1
    (3, 33, 5, 5, 17, 1, 1, 0),      # 1x1, non-multiple-of-16 channels
    (2, 7, 11, 13, 5, 5, 1, 2),      # generic-kernel template (5x5)
    (64, 6, 64, 64, 6, 3, 1, 1),     # PINN 6-channel conv at 64^2: >64 wgrad splits (two-level sum)
    (2, 5, 10, 11, 7, 3, 3, 1),      # stride 3, small: backward-data as one launch (MODE 1)
    (16, 128, 65, 65, 256, 3, 2, 0),  # NCSN++ FIR-down conv: backward-data by pixel class (MODE 3)
    (16, 128, 32, 32, 16, 3, 1, 1),  # PINN 16-channel conv: weight gradient on 16 x 256 tiles
]


@pytest.mark.parametrize("case", _IG_CASES)
def test_conv2d_igemm_fwd_dgrad_wgrad_vs_fp64(hip, case):
    """The implicit-GEMM kernels (forward + bias, backward-data, weight + bias gradient) vs
    float64 F.conv2d on the CPU; fp32 MFMA (exact products, k-ordered fma chain): error
    within 2e-5 of the output's magnitude (sums of up to ~2300 products; an indexing or
    padding error shows up as O(1))."""
    from op.conv import conv2d_igemm_raw, conv2d_input_igemm_raw, conv2d_weight_igemm_raw
    N, C, H, W, Co, k, s, p = case
    g = torch.Generator().manual_seed(sum(case))
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(Co, C, k, k, generator=g) / (C * k * k) ** 0.5
    b = torch.randn(Co, generator=g)
    xd, wd, bd = (t.double().requires_grad_() for t in (x, w, b))
    yref = F.conv2d(xd, wd, bd, s, p)
    gy = torch.randn(yref.shape, generator=g)
    gx_ref, gw_ref, gb_ref = torch.autograd.grad(yref, (xd, wd, bd), gy.double())

    def close(got, ref, what):
        ref = ref.detach()
        tol = 2e-5 * max(1.0, float(ref.abs().max()))
        err = float((got.double().cpu() - ref).abs().max())
        assert err <= tol, f"{what}: {err} > {tol}"

    y = conv2d_igemm_raw(x.to(hip), w.to(hip), b.to(hip), s, p)
    close(y, yref, "forward")
    gx = conv2d_input_igemm_raw(x.shape, w.to(hip), gy.to(hip), s, p)
    close(gx, gx_ref, "dgrad")
    dw, db = conv2d_weight_igemm_raw(x.to(hip), w.shape, gy.to(hip), s, p, bias_grad=True)
    close(dw, gw_ref, "wgrad")
    close(db, gb_ref, "bias grad")
    dw2, none = conv2d_weight_igemm_raw(x.to(hip), w.shape, gy.to(hip), s, p, bias_grad=False)
    assert none is None and torch.equal(dw2, dw)


@pytest.mark.parametrize("case", [
    # kind, N1, N2, Cin, H, W, Cout, k, stride, pad
    ("wino", 8, 8, 32, 16, 16, 32, 3, 1, 1),      # PINN pyramid conv, both sources B = 8
    ("wino", 4, 6, 64, 8, 8, 48, 3, 1, 1),        # 8-wide images (pair form), uneven sources
    ("wino", 3, 5, 32, 32, 32, 16, 3, 1, 1),      # odd first source, 32^2
    ("igemm", 8, 8, 16, 64, 64, 16, 3, 1, 1),     # PINN 16-channel conv at 64^2 (16 x 256 tiles)
    ("igemm", 5, 3, 49, 8, 8, 128, 3, 1, 1),      # corr_conv first conv (Cin 49)
    ("igemm", 4, 4, 16, 32, 32, 32, 3, 2, 1),     # stride-2 pyramid conv
    ("igemm", 2, 3, 6, 9, 9, 4, 4, 2, 1),         # k4 s2 (ConvTranspose class)
])
def test_wgrad_two_sources_match_sum_vs_fp64(hip, case):
    """bpk_conv3x3_wino_wgrad2_f32 / bpk_conv2d_igemm_wgrad2_f32 (the deferred weight gradients
    of op.conv.deferred_weight_grads): dw = wgrad(x1, gy1) + wgrad(x2, gy2) in one launch, db =
    the first source's bias gradient -- vs float64 autograd on the CPU, within 2e-5 of the
    gradient's magnitude (an image of the wrong source, or the second source's bias column,
    shows up as O(1))."""
    from op.conv import conv2d_weight_igemm2_raw, conv3x3_wgrad2_raw
    kind, N1, N2, C, H, W, Co, k, s, p = case
    g = torch.Generator().manual_seed(11 + sum(case[1:]))
    x1, x2 = torch.randn(N1, C, H, W, generator=g), torch.randn(N2, C, H, W, generator=g)
    w = (torch.randn(Co, C, k, k, generator=g) / (C * k * k) ** 0.5).double().requires_grad_()
    b = torch.zeros(Co, dtype=torch.float64, requires_grad=True)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    gy1, gy2 = torch.randn(N1, Co, Ho, Wo, generator=g), torch.randn(N2, Co, Ho, Wo, generator=g)
    y1 = F.conv2d(x1.double(), w, b, s, p)
    y2 = F.conv2d(x2.double(), w, None, s, p)
    gw_ref, gb_ref = torch.autograd.grad((y1 * gy1.double()).sum() + (y2 * gy2.double()).sum(),
                                         (w, b))
    d = [t.to(hip) for t in (x1, gy1, x2, gy2)]
    if kind == "wino":
        dw, db = conv3x3_wgrad2_raw(*d, tuple(w.shape), bias_grad=True)
    else:
        dw, db = conv2d_weight_igemm2_raw(*d, tuple(w.shape), s, p, bias_grad=True)
    for got, ref, what in ((dw, gw_ref, "dw"), (db, gb_ref, "db")):
        tol = 2e-5 * max(1.0, float(ref.abs().max()))
        err = float((got.double().cpu() - ref).abs().max())
        assert err <= tol, f"{what}: {err} > {tol}"


def test_deferred_weight_grads_match_autograd(hip):
    """op.conv.deferred_weight_grads around the backward of a PINN-shaped double backward
    (a first-order input gradient with create_graph, then a loss of it and of the output):
    every parameter's .grad matches autograd's per-node weight gradients (the same sums up to
    the order of the additions), through Winograd 3x3 convs, a general stride-2 conv, a conv
    transpose, 1x1 convs (PressureNet's shortcuts: the adjoint's transposed weight) and
    PressureNet ResidualBlocks in their fan-out form (the skip gradient added inside the
    InstanceNorm backward kernel); the accumulation into an existing .grad keeps autograd's
    semantics."""
    from models import layers
    from op import conv as conv_op
    from op.fused_act import leaky_relu
    torch.manual_seed(3)
    net = torch.nn.ModuleList([
        layers.Conv2d(16, 32, 3, padding=1), layers.Conv2d(32, 32, 3, padding=1),
        layers.Conv2d(32, 16, 3, stride=2, padding=1),
        layers.ConvTranspose2d(16, 16, 2, stride=2),
        layers.ResidualBlock(16, 32), layers.ResidualBlock(32, 32),   # 1x1 shortcut, identity
        layers.Conv2d(32, 8, 1)]).to(hip)
    x = torch.randn(8, 16, 16, 16, device=hip, requires_grad=True)

    def run(defer, twice=False):
        for q in net.parameters():
            q.grad = None
        prev = layers._IN_FANOUT
        layers._IN_FANOUT = defer  # the ResidualBlocks' fan-out form with it
        try:
            for _ in range(2 if twice else 1):
                h = x
                for i, m in enumerate(net):
                    h = m(h)
                    if i < 3:
                        h = leaky_relu(h, 0.1)
                gx, = torch.autograd.grad(h.sum(), x, create_graph=True)
                loss = (gx ** 2).sum() + (h ** 2).sum()
                with conv_op.deferred_weight_grads(defer):
                    loss.backward(inputs=list(net.parameters()))
        finally:
            layers._IN_FANOUT = prev
        return [q.grad.clone() for q in net.parameters()]

    ref = run(False)
    got = run(True)
    # absolute floor from the largest gradient: a conv bias in front of an InstanceNorm has an
    # analytically zero gradient, whose computed value is rounding noise either way
    scale = max(float(r.abs().max()) for r in ref)
    for a, r in zip(got, ref):
        assert torch.allclose(a, r, rtol=1e-5, atol=1e-5 * scale), float((a - r).abs().max())
    got2 = run(True, twice=True)  # .grad already set: the deferred gradients add into it
    for a, r in zip(got2, ref):
        assert torch.allclose(a, 2 * r, rtol=1e-5, atol=2e-5 * scale)


@pytest.mark.parametrize("case", [
    # N, Cin, H, W, Cout, K
    (2, 5, 9, 13, 1, 3),       # odd sizes, bands ragged
    (3, 16, 64, 64, 4, 3),     # PINN head shape
    (2, 7, 8, 300, 2, 3),      # W > 256: one pixel per thread per row step
    (2, 3, 5, 7, 3, 1),        # 1x1
    (1, 4, 1, 1, 2, 3),        # 1 x 1 image: every tap but the centre reads padding
    (4, 128, 32, 32, 1, 3),    # NCSN++ conv_out shape class (128 -> 1)
])
def test_conv2d_wgrad_small_cout_vs_fp64(hip, case):
    """Weight + bias gradient of a conv into Cout <= 4 channels (csrc/conv_small.hip streaming
    kernel) vs float64 autograd on the CPU: within 2e-5 of the gradient's magnitude;
    deterministic (two calls bit-identical)."""
    from op.conv import conv2d_weight_small_cout_raw
    N, C, H, W, Co, K = case
    g = torch.Generator().manual_seed(sum(case))
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(Co, C, K, K, generator=g)
    gy = torch.randn(N, Co, H, W, generator=g)
    xd, wd, bd = x.double(), w.double().requires_grad_(), torch.zeros(Co, dtype=torch.float64, requires_grad=True)
    y = F.conv2d(xd, wd, bd, 1, K // 2)
    gw_ref, gb_ref = torch.autograd.grad(y, (wd, bd), gy.double())
    dw, db = conv2d_weight_small_cout_raw(x.to(hip), w.shape, gy.to(hip), bias_grad=True)
    for got, ref, what in ((dw, gw_ref, "dw"), (db, gb_ref, "db")):
        tol = 2e-5 * max(1.0, float(ref.abs().max()))
        err = float((got.double().cpu() - ref).abs().max())
        assert err <= tol, f"{what}: {err} > {tol}"
    dw2, none = conv2d_weight_small_cout_raw(x.to(hip), w.shape, gy.to(hip), bias_grad=False)
    assert none is None and torch.equal(dw2, dw)


@pytest.mark.parametrize("cin", [1, 4])
def test_conv2d_input_select_small_cin_candidates(hip, cin, monkeypatch):
    """Backward-data into <= 4 channels: both candidates of the timed choice (the small-Cout
    kernel on the flipped / transposed filter, and igemm) vs float64 conv2d_input."""
    from op import conv
    g = torch.Generator().manual_seed(cin)
    xshape = (3, cin, 16, 20)
    w = torch.randn(64, cin, 3, 3, generator=g) / 24
    gy = torch.randn(3, 64, 16, 20, generator=g)
    ref = torch.nn.grad.conv2d_input(xshape, w.double(), gy.double(), 1, 1)
    for c in (0, 1):
        monkeypatch.setattr(conv, "_CHOICE", {("dsc", xshape, tuple(w.shape), (1, 1), (1, 1)): c})
        got = conv.conv2d_input_select(xshape, w.to(hip), gy.to(hip), 1, 1)
        err = float((got.double().cpu() - ref).abs().max())
        assert err <= 2e-5 * max(1.0, float(ref.abs().max())), (c, err)


@pytest.mark.parametrize("k,stride,pad,cin,cout,hw", [(3, 2, 1, 3, 16, 12), (3, 1, 1, 49, 32, 4),
                                                       (2, 2, 0, 8, 8, 6), (1, 1, 0, 5, 1, 7)])
def test_conv2d_general_igemm_double_backward(hip, k, stride, pad, cin, cout, hw):
    """conv2d_general on the implicit-GEMM kernels: forward, first derivatives with
    create_graph and a second derivative w.r.t. (x, w, b) equal F.conv2d's (fp32 on the
    device, both sides), as the PINN residual takes them."""
    from op.conv import conv2d_general
    g = torch.Generator().manual_seed(k * 7 + cin)
    x0 = torch.randn(2, cin, hw, hw + 1, generator=g).to(hip)
    w0 = (torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5).to(hip)
    b0 = torch.randn(cout, generator=g).to(hip)

    def second(fn):
        x, w, b = (t.clone().requires_grad_() for t in (x0, w0, b0))
        y = fn(x, w, b)
        (gx,) = torch.autograd.grad((y ** 2).sum(), x, create_graph=True)
        loss = (gx * torch.sin(x)).sum() + y.mean()
        return [y.detach()] + list(torch.autograd.grad(loss, (x, w, b)))

    got = second(lambda x, w, b: conv2d_general(x, w, b, stride, pad))
    with torch.backends.cudnn.flags(enabled=False):
        ref = second(lambda x, w, b: F.conv2d(x, w, b, stride, pad))
    for a, r in zip(got, ref):
        tol = 1e-4 * max(1.0, float(r.abs().max()))
        assert float((a - r).abs().max()) <= tol


@pytest.mark.parametrize("cin,cout,k,s,p,op,groups", [(2, 2, 4, 2, 1, 0, 2), (32, 16, 2, 2, 0, 0, 1),
                                                       (4, 6, 3, 2, 1, 1, 1)])
def test_conv_transpose2d_general_vs_torch(hip, cin, cout, k, s, p, op, groups):
    """layers.ConvTranspose2d (the dgrad kernel as the transposed conv, groups through a
    block-diagonal dense weight): forward, input / weight / bias gradients and a second
    derivative equal torch's ConvTranspose2d."""
    import copy
    import torch.nn as nn
    from models import layers
    torch.manual_seed(cin * 10 + k)
    ref = nn.ConvTranspose2d(cin, cout, k, s, p, op, groups=groups).to(hip)
    mod = layers.ConvTranspose2d(cin, cout, k, s, p, op, groups=groups).to(hip)
    mod.load_state_dict(copy.deepcopy(ref.state_dict()))
    x0 = torch.randn(3, cin, 5, 7, device=hip)
    outs = []
    for m in (mod, ref):
        x = x0.clone().requires_grad_()
        y = m(x)
        (gx,) = torch.autograd.grad((y ** 2).sum(), x, create_graph=True)
        loss = (gx * x).sum() + y.sum()
        outs.append([y.detach()] + list(torch.autograd.grad(loss, [x] + list(m.parameters()))))
    for a, r in zip(*outs):
        assert a.shape == r.shape
        assert float((a - r).abs().max()) <= 1e-4 * max(1.0, float(r.abs().max()))


# ------------------------------------------------------------------ InstanceNorm + ELU

@pytest.mark.parametrize("shape", [(4, 16, 64, 64), (4, 128, 4, 4), (3, 5, 2, 2), (2, 3, 7, 5),
                                   (1, 1, 1, 1), (2, 8, 32, 32), (2, 4, 24, 20), (1, 3, 50, 60),
                                   (1, 2, 90, 50)])
def test_instance_norm_elu_matches_oracle(hip, shape):
    """csrc/instance_norm.hip forward / backward / double backward vs the float64 numpy
    restatement (pinned against torch's CPU composite in tests/test_oracle.py).  fp32:
    1e-5 relative to max|ref| (per-plane reductions in a different order)."""
    from oracle import instance_norm_ref as inr
    from op.norm_act import instance_norm_act
    g = torch.Generator().manual_seed(11)
    x = torch.randn(*shape, generator=g) * 2 + 0.3
    dy = torch.randn(*shape, generator=g)
    v = torch.randn(*shape, generator=g)
    xd = x.to(hip).requires_grad_()
    dyd = dy.to(hip).requires_grad_()
    y = instance_norm_act(xd)
    (dx,) = torch.autograd.grad(y, xd, dyd, create_graph=True)
    gdy, gx = torch.autograd.grad(dx, (dyd, xd), v.to(hip))

    def close(a, ref, tol=1e-5):
        ref = np.asarray(ref)
        err = np.abs(a.detach().cpu().double().numpy() - ref).max() / max(np.abs(ref).max(), 1e-6)
        assert err <= tol, err

    xn, dyn, vn = x.double().numpy(), dy.double().numpy(), v.double().numpy()
    close(y, inr.forward(xn))
    close(dx, inr.backward(dyn, xn))
    o_gdy, o_gx = inr.double_backward(vn, dyn, xn)
    close(gdy, o_gdy)
    close(gx, o_gx, 5e-5 if shape[-1] * shape[-2] > 1 else 1e-5)


def test_instance_norm_elu_gradgradcheck_and_third_order_refused(hip):
    from op.norm_act import instance_norm_act
    torch.manual_seed(5)
    x = torch.randn(2, 3, 4, 5, dtype=torch.float64, device=hip, requires_grad=True)
    f = lambda a: instance_norm_act(a[:, :, 1:])  # non-contiguous input, as a slice
    assert torch.autograd.gradcheck(f, (x,))
    assert torch.autograd.gradgradcheck(f, (x,))
    # a plane of 300 elements: the workgroup-per-plane kernels (257..4096)
    x3 = torch.randn(1, 2, 15, 20, dtype=torch.float64, device=hip, requires_grad=True)
    assert torch.autograd.gradcheck(instance_norm_act, (x3,))
    assert torch.autograd.gradgradcheck(instance_norm_act, (x3,))
    y = f(x)
    (dx,) = torch.autograd.grad(y.sum(), x, create_graph=True)
    (ddx,) = torch.autograd.grad((dx ** 2).sum(), x, create_graph=True)
    with pytest.raises(RuntimeError):
        ddx.sum().backward()


@pytest.mark.parametrize("shape", [(2, 3, 4, 5), (1, 2, 15, 20), (2, 8, 32, 32)])
def test_instance_norm_elu_fanout(hip, shape):
    """instance_norm_act_fanout(x) = (act(IN(x)), x) with the skip's gradient added inside the
    backward kernel: float64 gradcheck / gradgradcheck of (y, x) -> any loss, and in float32
    the fused add (bpk_instance_norm_act_bwd_add_f32) bit-identical to the plain backward plus
    autograd's add, first and second order."""
    from op.norm_act import instance_norm_act, instance_norm_act_fanout
    torch.manual_seed(7)
    x = torch.randn(*shape, dtype=torch.float64, device=hip, requires_grad=True)
    w = torch.randn(*shape, dtype=torch.float64, device=hip)
    f = lambda a: instance_norm_act_fanout(a)[0] * 2 + instance_norm_act_fanout(a)[1] * w  # noqa
    assert torch.autograd.gradcheck(f, (x,))
    assert torch.autograd.gradgradcheck(f, (x,))
    xf = (torch.randn(*shape, device=hip) * 2 + 0.3).requires_grad_()
    g1, g2 = torch.randn(*shape, device=hip), torch.randn(*shape, device=hip)
    v = torch.randn(*shape, device=hip)

    def grads(fan):
        if fan:
            y, xs = instance_norm_act_fanout(xf)
        else:
            y, xs = instance_norm_act(xf), xf
        # one skip contribution: the fused add then sums the same two terms autograd does
        (dx,) = torch.autograd.grad((y * g1).sum() + (xs * g2).sum(), xf, create_graph=True)
        (ddx,) = torch.autograd.grad((dx * v).sum(), xf)
        return dx.detach(), ddx

    for a, b in zip(grads(True), grads(False)):
        assert torch.equal(a, b)


def test_instance_norm_elu_residual_block_matches_aten(hip, monkeypatch):
    """PressureNet's ResidualBlock with the fused kernels vs the same block on aten
    (BPK_IN_FUSED off): output, input derivative with create_graph, and the parameter
    gradients of a loss on that derivative (the PINN residual's pattern)."""
    from models import layers
    torch.manual_seed(2)
    blk = layers.ResidualBlock(16, 32).to(hip)
    x0 = torch.randn(4, 16, 16, 16, device=hip)
    outs = []
    for fused in (True, False):
        monkeypatch.setattr(layers, "_IN_FUSED", fused)
        blk.zero_grad()
        x = x0.clone().requires_grad_()
        y = blk(x)
        (gx,) = torch.autograd.grad((y ** 2).sum(), x, create_graph=True)
        (gx.square().sum() + y.sum()).backward()
        outs.append([y.detach(), gx.detach()] + [p.grad.detach().clone() for p in blk.parameters()])
    # outputs 1e-4; parameter gradients 1e-3 of max(|ref|, 1e-3 x the largest gradient):
    # conv1.bias feeds normalize2, so its exact gradient is zero and both sides hold rounding
    gmax = max(b.abs().max().item() for b in outs[1][2:])
    for i, (a, b) in enumerate(zip(*outs)):
        floor, tol = (1e-3 * gmax, 1e-3) if i >= 2 else (1e-6, 1e-4)
        err = (a - b).abs().max().item() / max(b.abs().max().item(), floor)
        assert err < tol, (i, err)


@pytest.mark.parametrize("B,C,P,scale", [(3, 256, 256, 1.0), (2, 64, 256, 0.125), (2, 32, 128, 0.3),
                                         (5, 96, 64, 1.0 / 96 ** 0.5), (64, 256, 256, 1 / 16),
                                         (8, 256, 256, 1 / 16)])
def test_fused_attention_matches_fp32_reference(hip, B, C, P, scale):
    """csrc/attention.hip (q^T k logits, row softmax and the PV product in one kernel) vs the
    reference's bmm + softmax + bmm in float64 (1e-5 relative to max|ref|): one workgroup per
    64 queries (B = 64, P = 64) and the key-split form with its combine launch (the small
    batches: 2 or 4 splits)."""
    from op.attention import attention, lib
    assert (lib.bpk_attention_workspace_bytes(B, C, P) > 0) == (B * P // 64 <= 128 and P >= 128)
    g = torch.Generator().manual_seed(B * C + P)
    qkv = torch.randn(B, 3, C, P, generator=g) * 0.5
    q, k, v = qkv[:, 0].double(), qkv[:, 1].double(), qkv[:, 2].double()
    w = torch.softmax(torch.bmm(q.transpose(1, 2), k) * scale, dim=-1)
    ref = torch.bmm(v, w.transpose(1, 2))
    out = attention(qkv.to(hip), scale).double().cpu()
    assert out.shape == (B, C, P)
    assert (out - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


@pytest.mark.parametrize("block", ["AttnBlockpp", "AttnBlock"])
def test_attention_block_fused_equals_bmm_path(hip, monkeypatch, block):
    """AttnBlockpp (NCSN++) and AttnBlock (the ddpm net of nc_ddpmpp / DPS, routed through the
    same stacked q/k/v GEMM) at inference with the fused attention kernel vs the same block on
    the bmm + softmax + bmm path (1e-5 relative); the fused kernel must actually run."""
    import models.layers as lay
    import models.layerspp as lpp
    from op import attention as attn_op
    g = torch.Generator().manual_seed(5)
    blk = (lpp.AttnBlockpp(256, skip_rescale=True, init_scale=0.1) if block == "AttnBlockpp"
           else lay.AttnBlock(256)).to(hip).eval()
    with torch.no_grad():
        for p in blk.parameters():
            p.add_(torch.randn(p.shape, generator=g).to(hip) * 0.05)
    x = torch.randn(4, 256, 16, 16, generator=g).to(hip)
    calls = []
    real = attn_op.attention
    monkeypatch.setattr(attn_op, "attention", lambda *a, **k: calls.append(1) or real(*a, **k))
    with torch.no_grad():
        fused = blk(x)
        assert calls, "the fused attention kernel did not run"
        monkeypatch.setattr(lpp, "_ATTN_FUSED", False)
        ref = blk(x)
    assert (fused - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


def test_fused_attention_rejects_bad_shapes(hip):
    from op.attention import attention
    with pytest.raises(RuntimeError, match="unsupported"):
        attention(torch.zeros(1, 3, 48, 100, device=hip), 1.0)
    with pytest.raises(RuntimeError, match="HIP"):
        attention(torch.zeros(1, 3, 32, 64), 1.0)


@pytest.mark.parametrize("mode", ["pre_stats", "pre_skip", "plain", "two_sources"])
def test_conv3x3_winograd_large_launch(hip, mode):
    """A launch with more workgroups than CUs on the 16-cin 8-wave kernel
    (wino_f23_k16_kernel; 4 x 128 -> 128 @ 128^2 = 512 workgroups) vs F.conv2d in fp32 (1e-5
    relative), incl. the GroupNorm+SiLU prologue with bias and partial statistics, the
    residual tail, the plain form and two input sources."""
    import torch.nn.functional as F
    from op.conv import conv3x3, conv3x3_fwd_raw, gn_partials
    g = torch.Generator().manual_seed(17)
    N, cin, cout, hw = 4, 128, 128, 128
    x = (torch.randn(N, cin, hw, hw, generator=g) * 1.5).to(hip)
    w = (torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)).to(hip)
    b = torch.randn(cout, generator=g).to(hip)
    st = torch.stack([torch.rand(N, cin, generator=g) + 0.5, torch.randn(N, cin, generator=g) * 0.3], -1).to(hip)
    skip = torch.randn(N, cout, hw, hw, generator=g).to(hip)
    with torch.no_grad():
        if mode == "plain":
            a = x
            out = conv3x3_fwd_raw(x, w, b)
        else:
            a = F.silu(x * st[..., 0, None, None] + st[..., 1, None, None])
            if mode == "pre_stats":
                out = conv3x3(x, w, b, pre=st, stats=True)
            elif mode == "pre_skip":
                out = conv3x3(x, w, b, skip=skip, div=2 ** 0.5, pre=st, stats=True)
            else:
                out = conv3x3_fwd_raw(x[:, :48].contiguous(), w, b, pre=st, stats=True,
                                      x2=x[:, 48:].contiguous())
        ref = F.conv2d(a, w, b, padding=1)
        if mode == "pre_skip":
            ref = (skip + ref) / 2 ** 0.5
    scale = ref.abs().max().item()
    assert (out - ref).abs().max().item() <= 1e-5 * scale
    if mode != "plain":
        part, R, cnt = gn_partials(out)
        m = out.reshape(N, cout, hw // 8, 8, hw // 16, 16).mean((3, 5)).reshape(N, cout, R)
        assert (part[..., 0] - m).abs().max().item() <= 1e-5 * scale


@pytest.mark.parametrize("mode", ["pre_stats", "pre_skip", "plain", "two_sources", "dgrad"])
@pytest.mark.parametrize("N,cin,cout,hw", [(8, 256, 256, 16), (8, 512, 256, 16), (8, 256, 256, 32),
                                           (2, 128, 256, 16), (3, 256, 128, 32)])
def test_conv3x3_winograd_split_k(hip, mode, N, cin, cout, hw):
    """The split-K form (bpk_conv3x3_wino_splitk_f32) that the small per-GPU batches of a
    batch-sharded run take at the 32^2 / 16^2 levels: the launch is split (workspace > 0), and
    output, residual tail, two-source input, backward-data and the GroupNorm partial statistics
    match F.conv2d / the statistics of the output (1e-5 relative)."""
    import torch.nn.functional as F
    from op.conv import conv3x3, conv3x3_fwd_raw, gn_partials, lib
    assert lib.bpk_conv3x3_wino_splitk_bytes(N, cin, cin, cout, hw, hw) > 0
    g = torch.Generator().manual_seed(N * 1000 + cin + hw)
    x = (torch.randn(N, cin, hw, hw, generator=g) * 1.5).to(hip)
    w = (torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)).to(hip)
    b = torch.randn(cout, generator=g).to(hip)
    st = torch.stack([torch.rand(N, cin, generator=g) + 0.5, torch.randn(N, cin, generator=g) * 0.3], -1).to(hip)
    skip = torch.randn(N, cout, hw, hw, generator=g).to(hip)
    with torch.no_grad():
        a = F.silu(x * st[..., 0, None, None] + st[..., 1, None, None])
        if mode == "plain":
            out, ref = conv3x3_fwd_raw(x, w, b), F.conv2d(x, w, b, padding=1)
        elif mode == "pre_stats":
            out, ref = conv3x3(x, w, b, pre=st, stats=True), F.conv2d(a, w, b, padding=1)
        elif mode == "pre_skip":
            out = conv3x3(x, w, b, skip=skip, div=2 ** 0.5, pre=st, stats=True)
            ref = (skip + F.conv2d(a, w, b, padding=1)) / 2 ** 0.5
        elif mode == "two_sources":
            out = conv3x3_fwd_raw(x[:, :48].contiguous(), w, b, pre=st, stats=True,
                                  x2=x[:, 48:].contiguous())
            ref = F.conv2d(a, w, b, padding=1)
        else:  # dx = conv(gy, flip_t(w)): the Winograd backward-data form
            gy = torch.randn(N, cout, hw, hw, generator=g).to(hip)
            out = conv3x3_fwd_raw(gy, w, ft=True)
            ref = torch.nn.grad.conv2d_input(x.shape, w, gy, padding=1)
    scale = ref.abs().max().item()
    assert (out - ref).abs().max().item() <= 1e-5 * scale
    if mode in ("pre_stats", "pre_skip", "two_sources"):
        part, R, cnt = gn_partials(out)
        m = out.reshape(N, cout, hw // 8, 8, hw // 16, 16).mean((3, 5)).reshape(N, cout, R)
        v = out.reshape(N, cout, hw // 8, 8, hw // 16, 16).var((3, 5), unbiased=False).reshape(N, cout, R)
        assert (part[..., 0] - m).abs().max().item() <= 1e-5 * scale
        assert (part[..., 1] / cnt - v).abs().max().item() <= 1e-4 * v.abs().max().item()


@pytest.mark.parametrize("N,cin,cout,h", [(128, 256, 256, 8), (16, 256, 256, 8), (2, 512, 256, 8),
                                          (6, 32, 128, 16)])
@pytest.mark.parametrize("mode", ["plain", "skip", "pre", "dgrad"])
def test_conv3x3_winograd_pair_form_8_wide(hip, mode, N, cin, cout, h):
    """The 16-cin kernel's pair form for 8-pixel-wide images (two images per 8 x 16 region:
    CIFAR-10's 8 x 8 level) -- plain, residual tail, GroupNorm+SiLU prologue and backward-data,
    with and without split-K (N = 16, 2 take the split), vs F.conv2d (1e-5 of max|ref|)."""
    import torch.nn.functional as F
    from op.conv import conv3x3, conv3x3_fwd_raw, lib, wino_pair_supported, wino_supported
    g = torch.Generator().manual_seed(N * 7 + cin + h)
    x = torch.randn(N, cin, h, 8, generator=g).to(hip)
    w = (torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)).to(hip)
    b = torch.randn(cout, generator=g).to(hip)
    assert wino_pair_supported(x, w) and not wino_supported(x, w)
    assert not lib.bpk_conv3x3_wino_pair_supported(N + 1, cin, cout, h, 8)  # odd N: igemm
    with torch.no_grad():
        if mode == "plain":
            out, ref = conv3x3_fwd_raw(x, w, b), F.conv2d(x, w, b, padding=1)
        elif mode == "skip":
            skip = torch.randn(N, cout, h, 8, generator=g).to(hip)
            out = conv3x3_fwd_raw(x, w, b, skip=skip, div=2 ** 0.5)
            ref = (skip + F.conv2d(x, w, b, padding=1)) / 2 ** 0.5
        elif mode == "pre":
            st = torch.stack([torch.rand(N, cin, generator=g) + 0.5,
                              torch.randn(N, cin, generator=g) * 0.3], -1).to(hip)
            out = conv3x3(x, w, b, pre=st)
            ref = F.conv2d(F.silu(x * st[..., 0, None, None] + st[..., 1, None, None]), w, b,
                           padding=1)
        else:
            wt = (torch.randn(cin, cout, 3, 3, generator=g) / (3 * cout ** 0.5)).to(hip)
            gy = torch.randn(N, cin, h, 8, generator=g).to(hip)  # conv(gy, flip_t(wt)): cin -> cout
            out = conv3x3_fwd_raw(gy, wt, ft=True)
            ref = torch.nn.grad.conv2d_input((N, cout, h, 8), wt, gy, padding=1)
    scale = ref.abs().max().item()
    assert (out - ref).abs().max().item() <= 1e-5 * scale


@pytest.mark.parametrize("N,cin,cout,h,w", [(2, 128, 128, 8, 16), (3, 256, 256, 16, 8),
                                             (1, 16, 128, 32, 32), (2, 64, 256, 4, 24)])
@pytest.mark.parametrize("with_bias", [True, False])
def test_conv3x3_up2_fused_nearest_upsample(hip, N, cin, cout, h, w, with_bias):
    """conv3x3(nearest_x2(x)) with the upsample read in the Winograd patch load (ddpm
    Upsample, reference layers.py:576-590) vs a float64 interpolate + direct conv; 2e-5 of
    max|ref| as the plain Winograd conv.  Gradients (x, w, b) vs torch autograd of
    interpolate + F.conv2d, 3e-5 of max|ref| as the Winograd backward test."""
    from op.conv import conv3x3_up2, up2_supported
    g = torch.Generator().manual_seed(N * 100 + cin + h)
    x = torch.randn(N, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    b = torch.randn(cout, generator=g) if with_bias else None
    xu = F.interpolate(x.double(), scale_factor=2, mode="nearest")
    ref = F.conv2d(xu, wt.double(), None if b is None else b.double(), padding=1)
    assert up2_supported(x.to(hip), wt.to(hip))
    out = conv3x3_up2(x.to(hip), wt.to(hip), None if b is None else b.to(hip)).double().cpu()
    assert out.shape == ref.shape
    assert (out - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()
    # autograd
    xg = x.to(hip).requires_grad_()
    wg = wt.to(hip).requires_grad_()
    bg = None if b is None else b.to(hip).requires_grad_()
    go = torch.randn(ref.shape, generator=g).to(hip)
    ins = (xg, wg) + (() if bg is None else (bg,))
    got = torch.autograd.grad(conv3x3_up2(xg, wg, bg), ins, go)
    exp = torch.autograd.grad(F.conv2d(F.interpolate(xg, scale_factor=2, mode="nearest"), wg, bg,
                                       padding=1), ins, go)
    for a, r in zip(got, exp):
        assert (a - r).abs().max().item() <= 3e-5 * r.abs().max().item()


def test_ddpm_upsample_module_fused_equals_unfused(hip, monkeypatch):
    """layers.Upsample(with_conv=True) takes the fused kernel and matches the interpolate +
    Conv_0 path it replaces (BPK_WINO_UP2=0 equivalent), eval and under autograd."""
    from models import layers
    from op import conv as conv_op
    torch.manual_seed(0)
    m = layers.Upsample(128, with_conv=True).to(hip)
    x = torch.randn(2, 128, 16, 16, device=hip)
    with torch.no_grad():
        fused = m(x)
        monkeypatch.setattr(conv_op, "_WINO_UP2", False)
        plain = m(x)
    assert fused.shape == (2, 128, 32, 32)
    assert (fused - plain).abs().max().item() <= 1e-5 * plain.abs().max().item()


@pytest.mark.parametrize("hw", [(64, 64), (7, 12), (33, 64), (64, 4)])
def test_upfirdn2d_fir_pad2_asymmetric_taps(hip, hw):
    """The 1:1 FIR with pad (2, 2) and an asymmetric random 4x4 kernel -- the flip of the
    true convolution is visible -- on 37 planes (every base alignment of the odd-pitch
    output; the rolling kernel's tail-column path for 2^k widths) vs the oracle."""
    from op import upfirdn2d
    from oracle.upfirdn2d_ref import upfirdn2d_np
    H, W = hw
    g = torch.Generator().manual_seed(7 * H + W)
    x = torch.randn(37, 1, H, W, generator=g)
    k = torch.randn(4, 4, generator=g).numpy().astype(np.float32)
    y = upfirdn2d(x.to(hip), torch.tensor(k, device=hip), pad=(2, 2)).cpu().numpy()
    ref = upfirdn2d_np(x.numpy(), k, (1, 1), (1, 1), (2, 2, 2, 2))
    assert y.shape == ref.shape == (37, 1, H + 1, W + 1)
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------ strided batched GEMM
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("batch,M,N,K", [(3, 37, 70, 19), (2, 256, 256, 256), (1, 64, 512, 128)])
def test_gemm_sb_strided_operands_vs_fp64(hip, ta, tb, batch, M, N, K):
    """bpk_gemm_sb_f32 with every transpose combination read through strides (no copies),
    ragged tiles, bias per column / per row and accumulation, vs float64 (1e-5 relative)."""
    from op.matmul import gemm_sb
    g = torch.Generator().manual_seed(batch * 7 + M + N + K)
    a = torch.randn(batch, K, M, generator=g).transpose(1, 2) if ta else torch.randn(batch, M, K, generator=g)
    b = torch.randn(batch, N, K, generator=g).transpose(1, 2) if tb else torch.randn(batch, K, N, generator=g)
    bn, bm = torch.randn(N, generator=g), torch.randn(M, generator=g)
    ref = torch.bmm(a.double(), b.double())
    scale = ref.abs().max().item()
    ad, bd = a.to(hip), b.to(hip)
    out = gemm_sb(ad, bd).cpu()
    assert (out.double() - ref).abs().max().item() <= 1e-5 * scale
    out = gemm_sb(ad, bd, bn.to(hip), 1, alpha=0.5).cpu()
    assert (out.double() - (0.5 * ref + bn.double())).abs().max().item() <= 1e-5 * scale
    c0 = torch.randn(batch, M, N, generator=g)
    acc = gemm_sb(ad, bd, bm.to(hip), 2, out=c0.to(hip)).cpu()
    want = c0.double() + ref + bm.double()[:, None]
    assert (acc.double() - want).abs().max().item() <= 1e-5 * want.abs().max().item()


def test_gemm_sb_rejects_mismatched_shapes(hip):
    """Batch sizes that are neither equal nor 1, a wrong `out` and a bias of the wrong length
    raise before any launch (mismatched batches read past the smaller operand)."""
    from op.matmul import gemm_sb
    a, b = torch.randn(2, 8, 4, device=hip), torch.randn(3, 4, 5, device=hip)
    with pytest.raises(RuntimeError, match="batch"):
        gemm_sb(a, b)
    with pytest.raises(RuntimeError, match="out"):
        gemm_sb(a, b[:2], out=torch.zeros(2, 8, 6, device=hip))
    with pytest.raises(RuntimeError, match="bias"):
        gemm_sb(a, b[:2], torch.zeros(4, device=hip), 1)
    assert gemm_sb(a, b[:1]).shape == (2, 8, 5)  # batch 1 broadcasts


def test_linear_native_gradients_vs_fp64(hip):
    """op.matmul.linear (nn.Linear on the native GEMM: the time-embedding MLP / Dense_0) --
    output, first and second derivatives w.r.t. x, W, b vs float64 torch (2e-5 relative)."""
    from op.matmul import linear
    g = torch.Generator().manual_seed(3)
    x0 = torch.randn(6, 4, 96, generator=g)
    w0 = torch.randn(160, 96, generator=g) / 10
    b0 = torch.randn(160, generator=g)
    go = torch.randn(6, 4, 160, generator=g)

    def run(fn, dev, dt):
        x, w, b = (t.to(dev, dt).requires_grad_() for t in (x0, w0, b0))
        y = fn(x, w, b)
        gx, gw, gb = torch.autograd.grad(y, (x, w, b), go.to(dev, dt), create_graph=True)
        s = (gx ** 2).sum() + (gw * gw.detach()).sum()
        hx, hw = torch.autograd.grad(s, (x, w))
        return [t.detach().double().cpu() for t in (y, gx, gw, gb, hx, hw)]
    got = run(linear, hip, torch.float32)
    ref = run(torch.nn.functional.linear, "cpu", torch.float64)
    for a, r in zip(got, ref):
        assert (a - r).abs().max().item() <= 2e-5 * r.abs().max().item()


def test_attention_block_training_on_native_gemm(hip, monkeypatch):
    """AttnBlockpp under autograd (training / DPS): q^T k and v w^T with their gradients on
    the native GEMM equal the torch.bmm path (output and gradients w.r.t. x and the NIN
    weights, 1e-5 relative)."""
    import models.layerspp as lpp
    from op import matmul
    g = torch.Generator().manual_seed(8)
    blk = lpp.AttnBlockpp(128, skip_rescale=True, init_scale=0.1).to(hip).train()
    with torch.no_grad():
        for p in blk.parameters():
            p.add_(torch.randn(p.shape, generator=g).to(hip) * 0.05)
    x0 = torch.randn(3, 128, 16, 16, generator=g).to(hip)
    go = torch.randn(3, 128, 16, 16, generator=g).to(hip)

    def run():
        x = x0.clone().requires_grad_()
        y = blk(x)
        grads = torch.autograd.grad(y, [x] + [blk.NIN_0.W, blk.NIN_1.W, blk.NIN_2.W], go)
        return [y.detach()] + list(grads)
    calls = []
    real = matmul.gemm_sb
    monkeypatch.setattr(matmul, "gemm_sb", lambda *a, **k: calls.append(1) or real(*a, **k))
    got = run()
    assert len(calls) >= 6, "the attention GEMMs did not run on the native kernel"
    monkeypatch.setattr(matmul, "supported", lambda *t: False)
    ref = run()
    for a, r in zip(got, ref):
        assert (a - r).abs().max().item() <= 1e-5 * r.abs().max().item()


def test_filter_batch_matches_per_weight_transforms(hip):
    """op.conv.FilterBatch: one launch transforms every 3x3 conv weight of a module (forward
    and flipped) bit-identically to the per-weight entries; inside active() filter_transform
    returns those buffers; refresh() after an in-place weight update re-transforms; convs
    through the batch == convs without it."""
    import torch.nn as nn
    from op import conv as conv_op
    torch.manual_seed(3)
    m = nn.Sequential(nn.Conv2d(16, 32, 3, padding=1), nn.Conv2d(32, 48, 3, padding=1),
                      nn.Conv2d(48, 16, 1), nn.Conv2d(49, 64, 3, padding=1),
                      nn.Conv2d(64, 64, 3, stride=2, padding=1)).to(hip)
    fb = conv_op.FilterBatch(m)
    assert fb.n == 4  # 16->32 and 32->48, forward + flipped; not 49->64 (49 channels), not 1x1 / stride 2
    fb.refresh()
    convs = [c for c in m if isinstance(c, nn.Conv2d)]
    for c in convs:
        for ft in (False, True):
            e = fb.map.get((c.weight.data_ptr(), ft))
            if e is not None:  # per-weight entry (outside the batch)
                assert torch.equal(e[1], conv_op.filter_transform(c.weight, ft)), (e[0], ft)
    with fb.active():
        assert conv_op.filter_transform(m[0].weight) is fb.map[(m[0].weight.data_ptr(), False)][1]
        # the conv paths pass detached views of the parameter
        assert conv_op.filter_transform(m[1].weight.detach(), True) is \
            fb.map[(m[1].weight.data_ptr(), True)][1]
    with torch.no_grad():
        m[0].weight.mul_(1.5)
    fb.refresh()
    U0 = fb.map[(m[0].weight.data_ptr(), False)][1]
    assert torch.equal(U0, conv_op.filter_transform(m[0].weight))
    x = torch.randn(2, 16, 16, 16, device=hip)
    with conv_op.batched_filters(m):
        y1 = conv_op.conv3x3(x, m[0].weight, m[0].bias)
    y0 = conv_op.conv3x3(x, m[0].weight, m[0].bias)
    assert torch.equal(y1, y0)


@pytest.mark.gpu
def test_eval_block_higher_order_autograd_opt_out(hip):
    """The fused GroupNorm+SiLU conv of eval-mode blocks is first-order only: a double
    backward through it raises; inside models.layers.higher_order_autograd() the block records
    the unfused composition and the second derivative (d/dx of |d/dx|^2) matches the unfused
    path bit for bit (same ops)."""
    import models.layers as layers
    import models.layerspp as lpp
    torch.manual_seed(0)
    blk = lpp.ResnetBlockBigGANpp(act=torch.nn.SiLU(), in_ch=64, out_ch=64, temb_dim=32,
                                  skip_rescale=True, init_scale=0., dropout=0.0).to(hip).eval()
    with torch.no_grad():
        for p in blk.parameters():
            p.add_(torch.randn_like(p) * 0.05)
    x0 = torch.randn(2, 64, 16, 16, device=hip)
    temb = torch.randn(2, 32, device=hip)

    def second():
        x = x0.clone().requires_grad_()
        g = torch.autograd.grad(blk(x, temb).square().sum(), x, create_graph=True)[0]
        return torch.autograd.grad(g.square().sum(), x)[0]
    with pytest.raises(RuntimeError):
        second()
    with layers.higher_order_autograd():
        a = second()
    old = layers._GN_CONV_AD, layers._SKIP_LINK, layers._GN_FANOUT
    layers._GN_CONV_AD, layers._SKIP_LINK, layers._GN_FANOUT = False, False, False
    try:
        b = second()
    finally:
        layers._GN_CONV_AD, layers._SKIP_LINK, layers._GN_FANOUT = old
    assert torch.isfinite(a).all() and torch.equal(a, b)
    assert layers._GN_CONV_AD and layers._GN_FANOUT  # restored


@pytest.mark.parametrize("kind,cin,cout,updown", [
    ("biggan", 64, 64, None), ("biggan", 64, 128, None), ("biggan", 64, 64, "down"),
    ("biggan", 64, 64, "up"), ("ddpmpp", 64, 64, None), ("ddpmpp", 64, 128, None)])
def test_gn_fanout_training_block_grads_bit_identical(hip, kind, cin, cout, updown):
    """Training-mode residual blocks with the GroupNorm fan-out (layers.gn_act_fanout: the
    skip's gradient -- identity, 1x1 projection, FIR resampling -- added inside the GroupNorm
    backward kernel): the block input's gradient and every parameter gradient bit-identical to
    the plain form, whose autograd adds the two gradients of the input."""
    from models import layers
    from models import layerspp as lpp
    torch.manual_seed(2)
    if kind == "biggan":
        blk = lpp.ResnetBlockBigGANpp(act=torch.nn.SiLU(), in_ch=cin, out_ch=cout, temb_dim=32,
                                      up=updown == "up", down=updown == "down", fir=True,
                                      dropout=0.0, skip_rescale=True).to(hip).train()
    else:
        blk = lpp.ResnetBlockDDPMpp(act=torch.nn.SiLU(), in_ch=cin, out_ch=cout, temb_dim=32,
                                    dropout=0.0, skip_rescale=True).to(hip).train()
    x0 = torch.randn(4, cin, 16, 16, device=hip)
    temb = torch.randn(4, 32, device=hip)

    def grads(fan):
        prev = layers._GN_FANOUT
        layers._GN_FANOUT = fan
        try:
            blk.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_()
            y = blk(x * 1.0, temb)
            (y * torch.linspace(-1, 1, y.numel(), device=hip).view_as(y)).sum().backward()
        finally:
            layers._GN_FANOUT = prev
        return [("y", y.detach()), ("x", x.grad)] + [(n, p.grad) for n, p in
                                                     blk.named_parameters()]

    for (name, a), (_, b) in zip(grads(True), grads(False)):
        assert a is not None and b is not None and torch.equal(a, b), name


@pytest.mark.parametrize("kind,cin,cout", [("biggan", 128, 256), ("ddpm", 256, 128),
                                           ("biggan", 128, 128)])
def test_gn_fanout_eval_fused_block_bit_identical(hip, kind, cin, cout):
    """Eval-mode blocks under autograd (DPS) on the fused GroupNorm+SiLU conv: with the fan-out
    (the 1x1 / conv shortcut's gradient of the block input added in the fused conv's GroupNorm
    backward, op.conv.gn_silu_conv3x3_ad(fanout=True)) the output, d/dx and every parameter
    gradient are bit-identical to the accumulation by autograd; identity-skip blocks keep the
    skip link."""
    import models.layers as layers
    import models.layerspp as lpp
    torch.manual_seed(1)
    if kind == "biggan":
        blk = lpp.ResnetBlockBigGANpp(act=torch.nn.SiLU(), in_ch=cin, out_ch=cout, temb_dim=64,
                                      skip_rescale=True, init_scale=0., dropout=0.0)
    else:
        blk = layers.ResnetBlockDDPM(act=torch.nn.SiLU(), in_ch=cin, out_ch=cout, temb_dim=64,
                                     dropout=0.0)
    blk = blk.to(hip).eval()
    with torch.no_grad():
        for p in blk.parameters():
            p.add_(torch.randn_like(p) * 0.05)
    x0 = torch.randn(4, cin, 16, 16, device=hip)
    temb = torch.randn(4, 64, device=hip)
    gout = torch.randn(4, cout, 16, 16, device=hip)

    def run(fan):
        prev = layers._GN_FANOUT
        layers._GN_FANOUT = fan
        try:
            blk.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_()
            y = blk(x * 1.0, temb)
            (y * gout).sum().backward()
        finally:
            layers._GN_FANOUT = prev
        return [y.detach(), x.grad] + [p.grad for p in blk.parameters()]

    for a, b in zip(run(True), run(False)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("N,C,G,H,W", [(4, 64, 32, 32, 32), (2, 128, 32, 8, 8), (3, 64, 16, 4, 4),
                                       (2, 96, 32, 16, 16), (2, 32, 8, 2, 2)])
def test_group_norm_backward_param_grads_deterministic(hip, N, C, G, H, W):
    """The resident GroupNorm+SiLU backward's gamma / beta gradients are summed in a fixed order
    (per-wave-slice butterflies, then the slices of a channel in order; a whole channel plane
    per lane segment for small planes): bit-identical over repeated runs, and within 2e-5 of
    the float64 autograd reference."""
    from op.norm_act import ACT_SILU, group_norm_act_f
    g = torch.Generator(device=hip).manual_seed(N * C + H)
    x = torch.randn(N, C, H, W, device=hip, generator=g)
    gam = torch.randn(C, device=hip, generator=g)
    bet = torch.randn(C, device=hip, generator=g)
    gy = torch.randn(N, C, H, W, device=hip, generator=g)

    def run():
        xs, ws, bs = (t.clone().requires_grad_() for t in (x, gam, bet))
        y = group_norm_act_f(xs, G, ws, bs, 1e-6, ACT_SILU)
        return torch.autograd.grad(y, (xs, ws, bs), gy)
    r1 = run()
    for _ in range(4):
        for a, b in zip(run(), r1):
            assert torch.equal(a, b)
    xd, wd, bd = (t.double().cpu().requires_grad_() for t in (x, gam, bet))
    yd = torch.nn.functional.silu(torch.nn.functional.group_norm(xd, G, wd, bd, 1e-6))
    ref = torch.autograd.grad(yd, (xd, wd, bd), gy.double().cpu())
    for a, r in zip(r1, ref):
        assert float((a.double().cpu() - r).abs().max()) <= 2e-5 * max(1.0, float(r.abs().max()))
