"""GPU parity of the score networks, PC sampler and train step against the reference
fixtures (tests/golden) and the CPU oracle."""
import numpy as np
import pytest
import torch

from conftest import load_golden, net_fixture, product_config, record_err
from oracle import nets_ref, score_sde_ref

pytestmark = pytest.mark.gpu

# fp32 tolerance for whole networks: MIOpen / hipBLASLt accumulate in a different order
# than the CPU reference (same dtype, different summation order)
NET_RTOL = 1e-4
# PC trajectories (N = 25, recorded noise) after the whole run, relative to max(1, max|ref|):
# measured 2e-7 .. 2e-6 on MI355X (gpurun_out/parity_errors.json, profiles/r02_parity_errors.json)
PC_RTOL = 2e-4


def _model(name, hip):
    import models  # noqa: F401
    from models import utils as mutils
    cfg, sd, x, labels, y = net_fixture(name)
    model = mutils.create_model(product_config(cfg, hip), wrap=False)
    model.load_state_dict({k: torch.tensor(v) for k, v in sd.items()}, strict=True)
    model.eval()
    return cfg, model, x, labels, y


def _close(a, b, rtol, what=None):
    scale = max(1.0, float(np.abs(b).max()))
    err = float(np.abs(a - b).max())
    if what:
        record_err(what, err / scale, rtol)
    assert err <= rtol * scale, f"max err {err:.3e} > {rtol:.1e} * {scale:.3e}"


@pytest.mark.parametrize("name", ["ncsnpp_a", "ncsnpp_b", "ncsnpp_c", "ddpm_a"])
def test_networks_match_reference_fixture(hip, name):
    cfg, model, x, labels, y = _model(name, hip)
    with torch.no_grad():
        out = model(torch.tensor(x, device=hip), torch.tensor(labels, device=hip))
    _close(out.cpu().numpy(), y, NET_RTOL, f"net {name}")


def test_ncsnpp_128_full_size_matches_cpu_oracle(hip):
    """The benchmark network (62.7M params, 128x128x1) against the oracle on CPU."""
    import models  # noqa: F401
    from configs.vp import nc_ncsnpp_128
    from models import utils as mutils
    torch.manual_seed(0)
    c = nc_ncsnpp_128.get_config()
    c.device = hip
    model = mutils.create_model(c, wrap=False).eval()
    with torch.no_grad():  # non-zero init everywhere (Conv_1 / NIN_3 start at zero)
        for p in model.parameters():
            p.add_(torch.randn_like(p) * 0.01)
    x = torch.rand(2, 1, 128, 128)
    t = torch.tensor([0.3, 0.9]) * 999
    with torch.no_grad():
        out = model(x.to(hip), t.to(hip)).cpu().numpy()
    params = nets_ref.init_params(model.state_dict())
    ref = nets_ref.forward(params, c, x, t).numpy()
    _close(out, ref, NET_RTOL, "ncsnpp 128 vs oracle")


def test_nc_ddpmpp_128_fused_blocks_match_unfused_and_cpu_oracle(hip, monkeypatch):
    """The literal nc_ddpmpp net (`ddpm`, 128x128x1) at inference: ResnetBlockDDPM on the
    GroupNorm+SiLU-prologue Winograd convs with the residual tail in Conv_1's epilogue and
    GroupNorm statistics from the producers' epilogues (models/layers.py) vs the unfused
    GroupNorm / conv / residual launches (BPK_DDPM_FUSED=0) and vs the oracle on CPU."""
    import models  # noqa: F401
    from configs.vp import nc_ddpmpp
    from models import layers
    from models import utils as mutils
    torch.manual_seed(0)
    c = nc_ddpmpp.get_config()
    c.device = hip
    model = mutils.create_model(c, wrap=False).eval()
    with torch.no_grad():  # non-zero init everywhere (Conv_1 starts at zero)
        for p in model.parameters():
            p.add_(torch.randn_like(p) * 0.01)
    x = torch.rand(2, 1, 128, 128)
    t = torch.tensor([3.0, 870.0])
    with torch.no_grad():
        fused = model(x.to(hip), t.to(hip)).cpu().numpy()
        monkeypatch.setattr(layers, "_DDPM_FUSED", False)
        plain = model(x.to(hip), t.to(hip)).cpu().numpy()
    _close(fused, plain, NET_RTOL, "nc_ddpmpp 128 fused vs unfused")
    params = nets_ref.init_params(model.state_dict())
    ref = nets_ref.forward(params, c, x, t).numpy()
    _close(fused, ref, NET_RTOL, "nc_ddpmpp 128 vs oracle")


@pytest.mark.parametrize("name", ["em_langevin", "rd_ald", "anc_none", "em_none"])
def test_pc_sampler_matches_reference_with_injected_noise(hip, name):
    """Fused PC engine, fed the reference's own noise draws, reproduces its samples."""
    import sampling
    import sde_lib
    from op import sde_kernels as K
    d = load_golden(f"pc_{name}.npz")
    cfg, model, *_ = _model(str(d["net"]), hip)
    sde = sde_lib.VPSDE(0.1, 20., int(d["N"]))
    draws = [torch.tensor(z) for z in d["draws"]]
    n_steps = int(d["n_steps"])
    pred, corr = str(d["predictor"]), str(d["corrector"])
    # map the reference's sequential draw order onto (step, draw-id) of the engine
    per_step = (n_steps if corr != "none" else 0) + (1 if pred != "none" else 0)
    order = [1 + j for j in range(n_steps if corr != "none" else 0)] + ([0] if pred != "none" else [])
    table = {}
    for i in range(int(d["N"])):
        for k, draw_id in enumerate(order):
            table[(i, draw_id)] = draws[i * per_step + k]
    eng = sampling.PCEngine(sde, tuple(d["prior"].shape), sampling.get_predictor(pred),
                            sampling.get_corrector(corr), float(d["snr"]), n_steps,
                            continuous=bool(d["continuous"]), device=hip,
                            noise_fn=lambda i, draw: table[(i, draw)])
    out, nfe = eng(model, x_init=torch.tensor(d["prior"]))
    assert nfe == int(d["nfe"])
    _close(out.cpu().numpy(), d["out"], PC_RTOL, f"pc {name}")


def test_pc_engine_graph_replay_equals_eager_and_is_shard_invariant(hip):
    import sampling
    import sde_lib
    cfg, model, *_ = _model("ncsnpp_a", hip)
    sde = sde_lib.VPSDE(0.1, 20., 25)
    prior = torch.randn(4, 1, 32, 32)
    mk = lambda graph, shape: sampling.PCEngine(sde, shape, sampling.EulerMaruyamaPredictor,
                                                sampling.LangevinCorrector, 0.075, 1,
                                                continuous=True, device=hip, seed=1234,
                                                use_graph=graph)
    eager = mk(False, (4, 1, 32, 32))
    graph = mk(True, (4, 1, 32, 32))
    xe, _ = eager.run(model, prior)
    xg, _ = graph.run(model, prior)
    assert graph.graph is not None, getattr(graph, "capture_error", "")
    assert torch.equal(xe, xg)
    # the step graph reads the cached Winograd filter transforms (op.conv.static_filters);
    # rewriting the weights in place after the capture (as EMA copy_to does) must reach the
    # replays through refresh_filters
    assert graph._filters, "no Winograd filter registered by the capture"
    with torch.no_grad():
        for p in model.parameters():
            if p.dim() == 4:
                p.mul_(1.05)
    xe2, _ = eager.run(model, prior)
    xg2, _ = graph.run(model, prior)
    assert not torch.equal(xe2, xe)
    assert torch.equal(xe2, xg2)


def test_fused_update_kernels_bit_exact_vs_cpu_formula(hip):
    """Same model output + same noise -> the fused EM / Langevin kernels reproduce the
    reference's float32 expressions bit for bit (FMA contraction is off in sampler.hip)."""
    import sampling
    import sde_lib
    from op import sde_kernels as K
    sde = sde_lib.VPSDE(0.1, 20., 1000)
    torch.manual_seed(0)
    B = 3
    x = torch.randn(B, 1, 8, 8)
    m = torch.randn(B, 1, 8, 8)
    z = torch.randn(B, 1, 8, 8)
    t = torch.ones(B) * 0.4567
    rows = sampling.coef_rows(sde, t, True, K.PRED_EM)
    # reference expression order (sampling.py:181-187, sde_lib.py:103-110, models/utils.py:159)
    std = sde.marginal_coef(t)[1]
    score = -m / std[:, None, None, None]
    dc, g = sde.coefficient(t)
    drift = dc[:, None, None, None] * x - g[:, None, None, None] ** 2 * score * 1.
    x_mean = x + drift * (-1. / sde.N)
    x_new = x_mean + g[:, None, None, None] * np.sqrt(1. / sde.N) * z
    xo, xm = torch.empty_like(x).to(hip), torch.empty_like(x).to(hip)
    K.predictor(K.PRED_EM, x.to(hip), m.to(hip), rows[None].to(hip),
                torch.zeros(1, dtype=torch.int32, device=hip), x_out=xo, x_mean=xm,
                noise=z.to(hip))
    assert torch.equal(xm.cpu(), x_mean) and torch.equal(xo.cpu(), x_new)


def test_philox_noise_is_standard_normal_and_shard_invariant(hip):
    from op import sde_kernels as K
    step = torch.tensor([7], dtype=torch.int32, device=hip)
    full = K.philox_normal((8, 4096), 99, step, 1, device=hip)
    half = K.philox_normal((4, 4096), 99, step, 1, sample_offset=4, device=hip)
    assert torch.equal(full[4:], half)
    v = full.double()
    assert abs(v.mean().item()) < 0.02 and abs(v.std().item() - 1) < 0.02


@pytest.mark.parametrize("name", ["dsm_ncsnpp", "dsm_fourier", "ddpm_discrete"])
def test_train_step_matches_reference(hip, name, monkeypatch):
    """One optimisation step (loss, grads, Adam update, EMA) with the reference's random draws."""
    import losses
    import sde_lib
    from models.ema import ExponentialMovingAverage
    d = load_golden(f"train_{name}.npz")
    cfg, model, *_ = _model(str(d["net"]), hip)
    c = product_config(net_fixture(str(d["net"]))[0], hip)
    model.train()
    rng = [(k.split("_", 1)[1], torch.tensor(d[k])) for k in sorted(
        (k for k in d.files if k.startswith("rng")), key=lambda s: int(s[3:].split("_")[0]))]
    it = iter(rng)

    def replay(kind):
        def f(*a, **kw):
            k, v = next(it)
            assert k == kind, (k, kind)
            return v.to(hip)
        return f

    monkeypatch.setattr(torch, "rand", replay("rand"))
    monkeypatch.setattr(torch, "randn_like", replay("randn_like"))
    monkeypatch.setattr(torch, "randint", replay("randint"))
    sde = sde_lib.VPSDE(c.model.beta_min, c.model.beta_max, c.model.num_scales)
    opt = losses.get_optimizer(c, model.parameters())
    ema = ExponentialMovingAverage(model.parameters(), decay=c.model.ema_rate)
    state = dict(optimizer=opt, model=model, ema=ema, step=int(d["step0"]))
    grads = {}
    real_step = opt.step

    def capture(*a, **kw):
        for k, p in model.named_parameters():
            if p.grad is not None:
                grads[k] = p.grad.detach().cpu().numpy()
        return real_step(*a, **kw)

    opt.step = capture
    step_fn = losses.get_step_fn(sde, train=True, optimize_fn=losses.optimization_manager(c),
                                 reduce_mean=c.training.reduce_mean,
                                 continuous=bool(d["continuous"]))
    loss = step_fn(state, torch.tensor(d["batch"], device=hip))
    assert abs(loss.item() - float(d["loss"])) <= 1e-4 * max(1.0, abs(float(d["loss"])))
    for k in grads:
        _close(grads[k], d["g:" + k], 2e-3)
    for k, p in model.named_parameters():
        _close(p.detach().cpu().numpy(), d["p1:" + k], 1e-4)


def test_eval_step_between_train_steps_leaves_training_unchanged(hip):
    """The eval step swaps the EMA weights in and out (ema.store / copy_to / restore); the
    Winograd filter transforms cached on each weight by the inference path (op/conv.py, keyed
    by the weight's version counter) must not survive the swap (`p.data.copy_`
    kept the version, so an inference forward after an eval step ran on the EMA weights'
    transforms).  The eval loss must be the EMA-weight model's, and an inference forward of
    the live weights after the eval step must equal the one before it, bit for bit."""
    import losses
    import models  # noqa: F401
    import sde_lib
    from configs.vp import nc_ncsnpp_128
    from models import utils as mutils
    from models.ema import ExponentialMovingAverage

    # the benchmark architecture at nf 32, 64^2: the inference convs run on the Winograd
    # kernel with the filter transform cached on the parameter
    c = nc_ncsnpp_128.get_config()
    c.model.nf = 32
    c.data.image_size = 64
    c.device = hip
    c.model.dropout = 0.0
    torch.manual_seed(0)
    model = mutils.create_model(c, wrap=False)
    with torch.no_grad():
        for p in model.parameters():
            p.add_(torch.randn_like(p) * 0.01)
    ema = ExponentialMovingAverage(model.parameters(), decay=c.model.ema_rate)
    with torch.no_grad():  # shadow weights clearly different from the live ones
        for s in ema.shadow_params:
            s.add_(torch.randn_like(s) * 0.05)
    sde = sde_lib.VPSDE(c.model.beta_min, c.model.beta_max, c.model.num_scales)
    evals = losses.get_step_fn(sde, False, reduce_mean=True, continuous=True)
    g = torch.Generator(device=hip).manual_seed(0)
    x = torch.rand(2, 1, 64, 64, device=hip, generator=g)
    t = torch.rand(2, device=hip, generator=g) * 0.9 + 0.05

    def infer():
        model.eval()
        with torch.no_grad():
            return model(x, t)

    y0 = infer()               # caches the live weights' transforms
    with torch.no_grad():      # an optimizer step: in-place update, version bump
        for p in model.parameters():
            p.add_(0.0)
    torch.manual_seed(99)
    loss_e = evals(dict(model=model, ema=ema, step=0), x)
    # the eval loss is the EMA-weight model's loss ...
    twin = mutils.create_model(c, wrap=False)  # fresh tensors: no cached transforms
    twin.load_state_dict(model.state_dict())
    with torch.no_grad():
        for p, s_ in zip([p for p in twin.parameters() if p.requires_grad], ema.shadow_params):
            p.copy_(s_)
    torch.manual_seed(99)
    loss_t = evals(dict(model=twin, ema=ExponentialMovingAverage(twin.parameters(), 0.9), step=0), x)
    assert abs(loss_e.item() - loss_t.item()) <= 1e-6 * abs(loss_t.item()), (loss_e.item(), loss_t.item())
    # ... and the next inference forward runs on the live weights again
    y1 = infer()
    assert torch.equal(y1, y0), float((y1 - y0).abs().max())
