"""Config-level golden fixtures: the REFERENCE run on CPU at each BASELINE.json config's
real architecture and resolution (reduced batch), so the HIP path is checked on the
networks it is benchmarked on, not only on tiny variants.

Run in the development container only (the reference does not travel):
    python tests/golden/make_golden_configs.py [name ...]

Weights are not stored: both sides fill every parameter with `conftest.seeded_fill_`
(numpy PCG64 per tensor, keyed by the parameter name), or -- PINN -- rebuild them with the
reference-identical seeded construction `conftest.build_pinn_weights`.  Large per-tensor
outputs (gradients, post-step parameters, EMA) keep the deterministic subset
`conftest.sample_idx`.  Dropout is set to 0 (the reference draws its masks from torch's
CPU generator inside F.dropout; parity needs identical draws).

Fixtures
  cfg_ddpmpp_cifar.npz   configs[0]: configs/vp/cifar10_ddpmpp_continuous.py (model `ddpm`,
                         32x32x3): forward at 4 labels + one continuous DSM train step at
                         step 2500 (B = 4, recorded t / z draws)
  cfg_ncsnpp_cifar.npz   configs[1]: configs/vp/cifar10_ncsnpp_continuous.py (32x32x3):
                         the same
  cfg_ncsnpp128_pc.npz   configs[2]: NCSN++ 128x128x1 (nc_ncsnpp_128), EM + Langevin PC
                         sampler (snr 0.075), continuous VP-SDE with N = 25, B = 2, every
                         noise draw recorded (50 score evaluations per sample)
  cfg_ncddpmpp128_pc.npz configs[2] literal variant: configs/vp/nc_ddpmpp.py at 128x128
                         (model `ddpm`, discrete, ancestral_sampling + none), N = 25, B = 1
  cfg_dps256.npz         configs[4]: configs/inverse/nc_ddpmpp_inpaint_dps.py at 256x256
                         (model `ddpm`), B = 2: score-net forward, and the reference's DPS
                         `ode_func` drift (x0_hat, measurement-gradient, drift) at two t
  cfg_pinn64.npz         configs[3]: configs/pinn/pinn_pde.py as shipped (64x64, feature_nums
                         [16, 32, 64, 96, 128]), B = 2: forward, equation_mse, sensitivities,
                         parameter gradients, and one get_pinn_step_fn train step
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, REPO)

import conftest  # noqa: E402,F401  (puts the build on sys.path BEFORE the reference is inserted)
from make_golden import REF, _config_json, _install_stubs, _save  # noqa: E402


K_SUB = 64  # elements kept per tensor (conftest.sample_idx(n, K_SUB)) in the train fixtures


def _structure(cfg, model):
    """The reference config (JSON) and every parameter's shape: the CPU suite checks the
    build's config modules and networks against them (tests/test_host.py)."""
    import json
    shapes = {k: list(p.shape) for k, p in model.named_parameters()}
    return {"config_json": np.array(_config_json(cfg)),
            "param_shapes": np.array(json.dumps(shapes, sort_keys=True))}


class _Stop(Exception):
    pass


def _record_rng(torch, names):
    """Wrap torch.<name> for name in names; returns (log, restore)."""
    log, real = [], {n: getattr(torch, n) for n in names}

    def wrap(n):
        def f(*a, **k):
            v = real[n](*a, **k)
            log.append((n, v.clone()))
            return v
        return f

    for n in names:
        setattr(torch, n, wrap(n))

    def restore():
        for n in names:
            setattr(torch, n, real[n])
    return log, restore


def gen_train(name, cfg_module, seed):
    """Forward + one DSM train step of a CIFAR-10 config (configs[0] / configs[1])."""
    import torch

    import losses
    import sde_lib
    from conftest import seeded_fill_, sub
    from models import ema
    from models import utils as mutils
    cfg = cfg_module.get_config()
    cfg.model.dropout = 0.0
    cfg.device = torch.device("cpu")
    model = seeded_fill_(mutils.get_model(cfg.model.name)(cfg), seed)
    g = torch.Generator().manual_seed(seed)
    B, C, n = 4, cfg.data.num_channels, cfg.data.image_size
    batch = torch.rand(B, C, n, n, generator=g) * 2 - 1  # centered data (scaler)
    labels = torch.tensor([0.999, 250.0, 600.5, 998.0])
    model.eval()
    with torch.no_grad():
        y = model(batch, labels)
    model.train()
    sde = sde_lib.VPSDE(beta_min=cfg.model.beta_min, beta_max=cfg.model.beta_max,
                        N=cfg.model.num_scales)
    opt = losses.get_optimizer(cfg, model.parameters())
    em = ema.ExponentialMovingAverage(model.parameters(), decay=cfg.model.ema_rate)
    state = dict(optimizer=opt, model=model, ema=em, step=2500)
    step_fn = losses.get_step_fn(sde, train=True, optimize_fn=losses.optimization_manager(cfg),
                                 reduce_mean=cfg.training.reduce_mean,
                                 continuous=cfg.training.continuous, likelihood_weighting=False)
    grads = {}
    real_step = opt.step

    def capture(*a, **k):
        for kk, p in model.named_parameters():
            if p.grad is not None:
                grads[kk] = p.grad.detach().clone()
        return real_step(*a, **k)

    opt.step = capture
    torch.manual_seed(seed + 1)
    log, restore = _record_rng(torch, ["rand", "randn_like", "randint"])
    try:
        loss = step_fn(state, batch)
    finally:
        restore()
    arr = {"batch": batch.numpy(), "labels": labels.numpy(), "y": y.numpy(),
           "loss": np.array(loss.item(), np.float64), "step0": np.array(2500),
           "seed": np.array(seed), "config": np.array(cfg_module.__name__.split(".")[-1]),
           **_structure(cfg, model)}
    for i, (kind, v) in enumerate(log):
        arr[f"rng{i}_{kind}"] = v.numpy()
    for k, v in grads.items():
        arr["g:" + k] = sub(v.numpy(), K_SUB)
    for k, v in model.named_parameters():
        arr["p1:" + k] = sub(v.detach().numpy(), K_SUB)
    names = [k for k, p in model.named_parameters() if p.requires_grad]
    for k, s in zip(names, em.shadow_params):
        arr["ema:" + k] = sub(s.numpy(), K_SUB)
    _save(f"cfg_{name}.npz", **arr)


def gen_pc(name, cfg, seed, predictor, corrector, snr, n_steps, N, B):
    """A whole PC trajectory of the reference's get_pc_sampler with every draw recorded."""
    import torch

    import sampling
    import sde_lib
    from conftest import regen_draws, seeded_fill_
    from models import utils as mutils
    cfg.device = torch.device("cpu")
    model = seeded_fill_(mutils.get_model(cfg.model.name)(cfg), seed).eval()
    sde = sde_lib.VPSDE(beta_min=cfg.model.beta_min, beta_max=cfg.model.beta_max, N=N)
    shape = (B, cfg.data.num_channels, cfg.data.image_size, cfg.data.image_size)
    torch.manual_seed(seed + 1)
    prior = sde.prior_sampling(shape)
    fn = sampling.get_pc_sampler(sde, shape, sampling.get_predictor(predictor),
                                 sampling.get_corrector(corrector), lambda v: v, snr,
                                 n_steps=n_steps, probability_flow=False,
                                 continuous=cfg.training.continuous, denoise=True, eps=1e-3,
                                 device="cpu")
    draws = []
    real = torch.randn_like
    real_prior = sde.prior_sampling
    sde.prior_sampling = lambda s: prior.clone()

    def rec(t, *a, **k):
        z = real(t, *a, **k)
        draws.append(z.clone())
        return z

    torch.manual_seed(seed + 2)
    torch.randn_like = rec
    try:
        with torch.no_grad():
            out, nfe = fn(model)
    finally:
        torch.randn_like = real
        sde.prior_sampling = real_prior
    # the draws are torch's CPU generator after manual_seed(seed + 2), one randn of the
    # sample shape per draw: the test regenerates them (conftest.regen_draws) and checks
    # them against a stored head of every draw
    dr = torch.stack(draws)
    assert torch.equal(dr, regen_draws(seed + 2, len(draws), shape))
    _save(f"cfg_{name}.npz", prior=prior.numpy(), out=out.numpy(), nfe=np.array(nfe),
          draw_seed=np.array(seed + 2), n_draws=np.array(len(draws)),
          draws_head=dr.reshape(len(draws), -1)[:, :64].numpy(), N=np.array(N), snr=np.array(snr),
          n_steps=np.array(n_steps), continuous=np.array(bool(cfg.training.continuous)),
          predictor=np.array(predictor), corrector=np.array(corrector), seed=np.array(seed),
          **_structure(cfg, model))


def gen_dps256(seed=31):
    """DPS drift of the reference (inverse/conditional_sampling.py:100-169) at 256x256.

    The reference InpaintOperator materialises (N, HW, HW) diagonal matrices (65536^2 x 4 B =
    17 GB per sample at 256^2, operators.py:157-197), so the fixture passes a stand-in
    with the same call contract: keep_shape=False is the gather of the observed pixels in
    row-major order, exactly what bcmm(pL, x) computes with the reference's 0/1 pL
    (columns e_idx in increasing idx, operators.py:125-130, 170-172) -- the operator itself
    is pinned at 16x16 against the dense form (tests/test_pinn_host.py, dps.npz)."""
    import torch

    import sde_lib
    from configs.inverse import nc_ddpmpp_inpaint_dps
    from conftest import seeded_fill_
    from inverse import conditional_sampling as cs
    from models import utils as mutils
    cfg = nc_ddpmpp_inpaint_dps.get_config()
    cfg.data.image_size = 256
    cfg.device = torch.device("cpu")
    model = seeded_fill_(mutils.get_model(cfg.model.name)(cfg), seed).eval()
    B, n = 2, 256
    g = torch.Generator().manual_seed(seed)
    mask = (torch.rand(1, 1, n, n, generator=g) > 0.5).float()
    idx = torch.nonzero(mask.reshape(-1)).reshape(-1)
    origin = torch.rand(B, 1, n, n, generator=g)
    x = torch.randn(B, 1, n, n, generator=g)

    class GatherInpaint:
        def __call__(self, v, keep_shape=True, invert=False):
            assert not invert
            if keep_shape:
                return mask * v
            return v.reshape(v.shape[0], v.shape[1], -1)[:, :, idx]

    op = GatherInpaint()
    y0 = op(origin, keep_shape=False)
    sde = sde_lib.VPSDE(cfg.model.beta_min, cfg.model.beta_max, cfg.model.num_scales)
    obsv = sde_lib.LOBSVSDE(sde, y0, op)
    labels = torch.tensor([0.3, 0.8]) * 999
    with torch.no_grad():
        y = model(x, labels)
    funcs = []
    real_ivp = cs.integrate.solve_ivp
    real_randn_like = torch.randn_like
    draws = []

    def rec(v, *a, **k):
        z = real_randn_like(v, *a, **k)
        draws.append(z.clone())
        return z

    def grab(fun, *a, **k):
        funcs.append(fun)
        raise _Stop

    torch.manual_seed(seed + 1)
    torch.randn_like = rec
    cs.integrate.solve_ivp = grab
    try:
        sampler = cs.get_dps_sampler(cfg, obsv, (B, 1, n, n), eps=1e-3)
        try:
            sampler(model, z=x)
        except _Stop:
            pass
    finally:
        torch.randn_like = real_randn_like
        cs.integrate.solve_ivp = real_ivp
    t_probe = [0.9, 0.4]
    probes = np.stack([funcs[0](tp, x.numpy().reshape(-1).astype(np.float64))
                       for tp in t_probe]).astype(np.float32)
    # a short stretch of the reference's own RK45 solve at 256^2 (scipy solve_ivp on the
    # captured ODE function, the tolerances of the reference's get_solver): accepted steps,
    # nfev and the final state
    t_span = (0.5, 0.45)
    sol = real_ivp(funcs[0], t_span, x.numpy().reshape(-1).astype(np.float64), method="RK45",
                   rtol=1e-3, atol=1e-3)
    _save("cfg_dps256.npz", mask=mask.numpy(), origin=origin.numpy(), x=x.numpy(),
          labels=labels.numpy(), y=y.numpy(), obs_noise=draws[0].numpy(),
          t_probe=np.array(t_probe), probes=probes, variance=np.array(cfg.inverse.variance),
          seed=np.array(seed), solve_t_span=np.array(t_span), solve_t=sol.t,
          solve_y=sol.y[:, -1].astype(np.float64), solve_nfev=np.array(sol.nfev),
          **_structure(cfg, model))


def gen_pinn64():
    """configs/pinn/pinn_pde.py as shipped, B = 2 (make_golden_pinn.py's recipe at full size)."""
    import torch

    from make_golden_pinn import MaskOp, install_pinn_stand_ins
    install_pinn_stand_ins()  # before anything imports the reference's op.correlation
    import losses
    from configs.pinn import pinn_pde
    from conftest import build_pinn_weights, full_pinn_config, make_pinn_inputs, sub
    from models import ema as ref_ema
    from pinn_kalman.pinn import PINN
    c = full_pinn_config(pinn_pde.get_config)
    model = build_pinn_weights(PINN, c)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    f1, f2, x, y, t, target = make_pinn_inputs(c, 11)
    xr, yr, tr = (v.clone().requires_grad_() for v in (x, y, t))
    model.train()
    flows, pres = model(f1, f2, xr, yr, tr)
    eq7 = model.equation_mse(xr, yr, tr, flows[-1], pres, 10000000.0)
    model.zero_grad()
    eq50 = model.equation_mse(xr, yr, tr, flows[-1], pres, 50.0)
    gx, gy, gt = torch.autograd.grad(eq50, (xr, yr, tr), retain_graph=True)
    eq50.backward()
    arr = {"sdsub:" + k: sub(v.numpy()) for k, v in sd.items()}
    arr.update(_structure(c, model))
    arr.update(f1=f1.numpy(), f2=f2.numpy(), x=x.numpy(), y=y.numpy(), t=t.numpy(),
               target=target.numpy(), pres=pres.detach().numpy(), eq7=np.array(eq7.item()),
               eq50=np.array(eq50.item()), gx=gx.numpy(), gy=gy.numpy(), gt=gt.numpy(),
               n_flows=np.array(len(flows)))
    for i, fl in enumerate(flows):
        arr[f"flow{i}"] = fl.detach().numpy()
    for k, p in model.named_parameters():
        if p.grad is not None:
            arr["g:" + k] = sub(p.grad.numpy())
    # one PINN train step (losses.py:332-386) at step 50 from the same weights
    m = PINN(c)
    m.load_state_dict(sd)
    em = ref_ema.ExponentialMovingAverage(m.parameters(), decay=c.model.ema_rate)
    opt_f = losses.get_optimizer(c, m.flownet.parameters())
    opt_p = losses.get_optimizer(c, m.pressurenet.parameters(), 0.001)
    state = dict(optimizer=(opt_f, opt_p), model=m, ema=em, step=50)
    step_fn = losses.get_pinn_step_fn(c, train=True, optimize_fn=losses.optimization_manager(c))
    g = torch.Generator().manual_seed(111)
    n = c.data.image_size
    mask = (torch.rand(1, 1, n, n, generator=g) <= 0.9).float().expand(2, 1, n, n).contiguous()
    grads = {}
    for opt, net, pref in ((opt_f, m.flownet, "flownet."), (opt_p, m.pressurenet, "pressurenet.")):
        def capture(*a, _real=opt.step, _net=net, _pref=pref, **k):
            for kk, p in _net.named_parameters():
                if p.grad is not None:
                    grads[_pref + kk] = p.grad.detach().clone()
            return _real(*a, **k)
        opt.step = capture
    torch.manual_seed(211)
    log, restore = _record_rng(torch, ["randn_like"])
    try:
        out = step_fn(state, MaskOp(mask), (f1, f2, x.clone().requires_grad_(),
                                            y.clone().requires_grad_(),
                                            t.clone().requires_grad_(), target))
    finally:
        restore()
    arr.update(step_mask=mask.numpy(), step_losses=np.array([o.item() for o in out]),
               step1=np.array(state["step"]))
    for i, (_, z) in enumerate(log):
        arr[f"noise{i}"] = z.numpy()
    for k, v in grads.items():
        arr["sg:" + k] = sub(v.numpy())
    for k, v in m.named_parameters():
        arr["p1:" + k] = sub(v.detach().numpy())
    names = [k for k, p in m.named_parameters() if p.requires_grad]
    for k, s in zip(names, em.shadow_params):
        arr["ema:" + k] = sub(s.numpy())
    _save("cfg_pinn64.npz", **arr)


def main(which):
    if not os.path.isdir(REF):
        print(f"reference not found at {REF}; nothing to do")
        return
    sys.dont_write_bytecode = True
    _install_stubs()
    sys.path.insert(0, REF)
    import torch
    torch.set_num_threads(8)
    from configs.vp import cifar10_ddpmpp_continuous, cifar10_ncsnpp_continuous, nc_ddpmpp
    from models import ddpm, ncsnpp  # noqa: F401  (registers the models)
    jobs = {
        "ddpmpp_cifar": lambda: gen_train("ddpmpp_cifar", cifar10_ddpmpp_continuous, 101),
        "ncsnpp_cifar": lambda: gen_train("ncsnpp_cifar", cifar10_ncsnpp_continuous, 102),
        "ncsnpp128_pc": lambda: gen_pc("ncsnpp128_pc", _ncsnpp128(cifar10_ncsnpp_continuous),
                                       103, "euler_maruyama", "langevin", 0.075, 1, 25, 2),
        "ncddpmpp128_pc": lambda: gen_pc("ncddpmpp128_pc", _ncddpmpp128(nc_ddpmpp), 104,
                                         "ancestral_sampling", "none", 0.16, 1, 25, 1),
        # the whole N = 1000 trajectory of the benchmark configuration (2000 evaluations,
        # B = 1; ~25 min on 8 host threads)
        "ncsnpp128_pc_long": lambda: gen_pc("ncsnpp128_pc_long",
                                            _ncsnpp128(cifar10_ncsnpp_continuous), 105,
                                            "euler_maruyama", "langevin", 0.075, 1, 1000, 1),
        "dps256": gen_dps256,
        "pinn64": gen_pinn64,
    }
    for k in which or jobs:
        print(f"== {k}", flush=True)
        jobs[k]()


def _ncsnpp128(mod):
    """The benchmark network's config composed from reference pieces, as the build's
    configs/vp/nc_ncsnpp_128.py composes it: configs/default_nc_configs.py + the NCSN++
    model section of configs/vp/cifar10_ncsnpp_continuous.py at 128x128x1, continuous VP
    (N = 1000), EM + Langevin (snr 0.075)."""
    from configs import default_nc_configs
    c = default_nc_configs.get_default_configs()
    c.training.update(dict(sde="vpsde", continuous=True, reduce_mean=True, batch_size=64))
    c.sampling.update(dict(method="pc", predictor="euler_maruyama", corrector="langevin",
                           snr=0.075, n_steps_each=1))
    c.data.update(dict(image_size=128, num_channels=1, centered=False))
    c.model.update(dict(mod.get_config().model))
    c.model.update(dict(num_scales=1000, dropout=0.0))
    return c


def _ncddpmpp128(mod):
    c = mod.get_config()
    c.data.image_size = 128
    return c


if __name__ == "__main__":
    main(sys.argv[1:])
