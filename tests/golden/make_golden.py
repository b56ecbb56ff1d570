"""Generate golden fixtures by running the REFERENCE (/root/reference) on CPU.

Run in the development container only (the reference does not travel):
    python tests/golden/make_golden.py
Writes small .npz files next to this script.  Each fixture holds inputs and the
reference's outputs; nothing of the reference's source is stored.

Import recipe: the reference's hot-path modules import
on CPU once modules that are absent here and that are NOT on the arithmetic
path are stubbed: torchvision / imageio (datasets only), ml_collections
(ConfigDict -> attribute dict), bayesian_torch (B-PINN only), and
torch.utils.cpp_extension.load (the CUDA JIT build; CPU branches never call it).
`run_lib._get_sde` is restated below because run_lib needs absl/tensorboard.

Fixtures:
  upfirdn2d.npz          upfirdn2d_native fwd + input-grad on 12 (up, down, pad, k) cases
  sde_tables.npz         VPSDE/VESDE/subVPSDE tables, PC time grid + index tables (N=1000, 2000)
  timestep_embedding.npz get_timestep_embedding
  net_<name>.npz         tiny NCSN++ / DDPM variants: weights, inputs, outputs
  pc_<name>.npz          3-step PC samplers (N=25) with every noise draw recorded
  train_<name>.npz       one DSM / DDPM train step: t, z, loss, grads, Adam update, EMA
  fused_lrelu.npz        op.fused_leaky_relu CPU branch
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

REF = os.environ.get("BPK_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_stubs():
    import torch

    # the build package (put on sys.path by tests/conftest.py) must not shadow the
    # reference's modules -- its `inverse` is a namespace package, which loses to any
    # regular package of the same name further down the path
    sys.path[:] = [p for p in sys.path if os.path.basename(p.rstrip("/")) != "b-pinn-kalman-filter_amd"]
    import torch.utils.cpp_extension as ce

    ce.load = lambda *a, **k: types.SimpleNamespace()
    for name in ["torchvision", "torchvision.datasets", "torchvision.transforms",
                 "torchvision.transforms.functional", "torchvision.utils", "imageio",
                 "imageio.v2"]:
        sys.modules[name] = types.ModuleType(name)
    sys.modules["torchvision.transforms.functional"].InterpolationMode = types.SimpleNamespace(
        BILINEAR=2, NEAREST=0)
    bt = types.ModuleType("bayesian_torch")
    btm = types.ModuleType("bayesian_torch.models")
    btd = types.ModuleType("bayesian_torch.models.dnn_to_bnn")
    btd.get_kl_loss = lambda m: None
    btd.dnn_to_bnn = lambda m, p: None
    sys.modules.update({"bayesian_torch": bt, "bayesian_torch.models": btm,
                        "bayesian_torch.models.dnn_to_bnn": btd})

    class ConfigDict(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

        def __setattr__(self, k, v):
            self[k] = v

    mc = types.ModuleType("ml_collections")
    mc.ConfigDict = ConfigDict
    sys.modules["ml_collections"] = mc
    return ConfigDict


def _config_json(cfg):
    import json

    def plain(v):
        if isinstance(v, dict):
            return {k: plain(x) for k, x in v.items() if k != "device"}
        if isinstance(v, (tuple, list)):
            return [plain(x) for x in v]
        return v

    return json.dumps(plain(cfg), sort_keys=True)


def _save(name, **arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"wrote {name} ({os.path.getsize(path) / 1024:.1f} KiB)")


def main():
    if not os.path.isdir(REF):
        print(f"reference not found at {REF}; nothing to do")
        return
    sys.dont_write_bytecode = True
    ConfigDict = _install_stubs()
    sys.path.insert(0, REF)
    import torch

    torch.set_num_threads(4)
    import losses
    import sampling
    import sde_lib
    from models import ddpm, ema, layers, ncsnpp  # noqa: F401  (registers models)
    from models import utils as mutils
    from op import fused_act
    from op.upfirdn2d import upfirdn2d_native

    # ------------------------------------------------------------- upfirdn2d
    k4 = np.outer([1, 3, 3, 1], [1, 3, 3, 1]).astype(np.float32)
    k4 /= k4.sum()
    rng = np.random.default_rng(1234)
    kasym = rng.standard_normal((4, 3)).astype(np.float32)
    k3 = rng.standard_normal((3, 3)).astype(np.float32)
    k2 = np.ones((2, 2), np.float32) / 4
    cases = [  # (shape, kernel, up_x, up_y, down_x, down_y, px0, px1, py0, py1)
        ((2, 3, 16, 16), k4, 1, 1, 2, 2, 1, 1, 1, 1),        # NCSN++ down2
        ((2, 3, 8, 8), k4 * 4, 2, 2, 1, 1, 2, 1, 2, 1),      # NCSN++ up2
        ((2, 3, 8, 8), k4, 1, 1, 1, 1, 2, 2, 2, 2),          # conv_downsample FIR
        ((1, 2, 13, 9), k4, 1, 1, 2, 2, 1, 1, 1, 1),         # odd / non-square
        ((1, 2, 7, 11), k4 * 4, 2, 2, 1, 1, 2, 1, 2, 1),
        ((1, 2, 10, 10), kasym, 1, 1, 1, 1, 1, 2, 0, 3),     # asymmetric kernel, per-axis pad
        ((1, 2, 10, 12), k3, 2, 2, 1, 1, 1, 1, 1, 1),        # 3x3 up2
        ((1, 2, 12, 12), k2, 1, 1, 2, 2, 0, 0, 0, 0),        # 2x2 down2
        ((1, 1, 9, 9), kasym, 1, 1, 1, 1, -1, 2, 2, -1),     # negative pad (crop)
        ((1, 2, 6, 6), k4, 3, 3, 1, 1, 2, 2, 2, 2),          # generic up3
        ((1, 2, 15, 15), k4, 1, 1, 3, 3, 1, 1, 1, 1),        # generic down3
        ((1, 2, 8, 10), k3, 2, 1, 1, 2, 1, 1, 2, 0),         # mixed per-axis factors
    ]
    up = {}
    for ci, (shape, k, ux, uy, dx, dy, px0, px1, py0, py1) in enumerate(cases):
        x = torch.tensor(rng.standard_normal(shape).astype(np.float32), requires_grad=True)
        kt = torch.tensor(k)
        y = upfirdn2d_native(x, kt, ux, uy, dx, dy, px0, px1, py0, py1)
        g = torch.tensor(rng.standard_normal(tuple(y.shape)).astype(np.float32))
        (gx,) = torch.autograd.grad(y, x, g)
        up[f"c{ci}_x"] = x.detach().numpy()
        up[f"c{ci}_k"] = k
        up[f"c{ci}_params"] = np.array([ux, uy, dx, dy, px0, px1, py0, py1], np.int64)
        up[f"c{ci}_y"] = y.detach().numpy()
        up[f"c{ci}_g"] = g.numpy()
        up[f"c{ci}_gx"] = gx.numpy()
    up["n_cases"] = np.array(len(cases))
    _save("upfirdn2d.npz", **up)

    # ------------------------------------------------------------- SDE tables
    tabs = {}
    for N in (1000, 2000):
        vp = sde_lib.VPSDE(beta_min=0.1, beta_max=20., N=N)
        tabs[f"vp{N}_discrete_betas"] = vp.discrete_betas.numpy()
        tabs[f"vp{N}_alphas"] = vp.alphas.numpy()
        tabs[f"vp{N}_alphas_cumprod"] = vp.alphas_cumprod.numpy()
        tabs[f"vp{N}_sqrt_alphas_cumprod"] = vp.sqrt_alphas_cumprod.numpy()
        tabs[f"vp{N}_sqrt_1m_alphas_cumprod"] = vp.sqrt_1m_alphas_cumprod.numpy()
        ts = torch.linspace(vp.T, 1e-3, vp.N)
        tabs[f"vp{N}_timesteps"] = ts.numpy()
        idx, drift, diff, std, mean, label999 = [], [], [], [], [], []
        for i in range(N):
            vec = torch.ones(2) * ts[i]
            idx.append((vec * (vp.N - 1) / vp.T).long()[0].item())
            dc, gc = vp.coefficient(vec)
            drift.append(dc[0].item())
            diff.append(gc[0].item())
            m, s = vp.marginal_coef(vec)
            mean.append(m[0].item())
            std.append(s[0].item())
            label999.append((vec * 999)[0].item())
        tabs[f"vp{N}_index"] = np.array(idx, np.int64)
        tabs[f"vp{N}_drift_coef"] = np.array(drift, np.float32)
        tabs[f"vp{N}_diffusion"] = np.array(diff, np.float32)
        tabs[f"vp{N}_marginal_mean"] = np.array(mean, np.float32)
        tabs[f"vp{N}_marginal_std"] = np.array(std, np.float32)
        tabs[f"vp{N}_labels999"] = np.array(label999, np.float32)
    class _ConcreteVE(sde_lib.VESDE):  # the reference VESDE is abstract (no marginal_coef)
        def marginal_coef(self, t):
            raise NotImplementedError

    ve = _ConcreteVE(sigma_min=0.01, sigma_max=50., N=1000)
    tabs["ve1000_discrete_sigmas"] = ve.discrete_sigmas.numpy()
    tv = torch.linspace(1e-3, 1., 37)
    tabs["ve_t"] = tv.numpy()
    tabs["ve_coef_diffusion"] = ve.coefficient(tv)[1].numpy()
    tabs["ve_marginal_std"] = ve.marginal_prob(torch.zeros(37, 1, 1, 1), tv)[1].numpy()
    tabs["ve_discretize_G"] = ve.discretize(torch.zeros(37, 1, 1, 1), tv)[1].numpy()
    sv = sde_lib.subVPSDE(beta_min=0.1, beta_max=20., N=1000)
    tabs["subvp_t"] = tv.numpy()
    tabs["subvp_drift"] = sv.coefficient(tv)[0].numpy()
    tabs["subvp_diffusion"] = sv.coefficient(tv)[1].numpy()
    tabs["subvp_mean"] = sv.marginal_coef(tv)[0].numpy()
    tabs["subvp_std"] = sv.marginal_coef(tv)[1].numpy()
    _save("sde_tables.npz", **tabs)

    # ------------------------------------------------------------- timestep embedding
    te = {}
    tt = torch.tensor([0., 1., 17.5, 250., 998.999, 999.], dtype=torch.float32)
    for dim in (8, 16, 33, 128):
        te[f"dim{dim}"] = layers.get_timestep_embedding(tt, dim).numpy()
    te["t"] = tt.numpy()
    _save("timestep_embedding.npz", **te)

    # ------------------------------------------------------------- tiny networks
    def base_config():
        c = ConfigDict()
        c.training = ConfigDict(continuous=True, batch_size=4, reduce_mean=True,
                                likelihood_weighting=False, sde="vpsde")
        c.sampling = ConfigDict(method="pc", predictor="euler_maruyama", corrector="langevin",
                                snr=0.075, n_steps_each=1, noise_removal=True,
                                probability_flow=False)
        c.data = ConfigDict(image_size=32, num_channels=1, centered=False)
        c.model = ConfigDict(name="ncsnpp", scale_by_sigma=False, ema_rate=0.9999,
                             normalization="GroupNorm", nonlinearity="swish", nf=16,
                             ch_mult=(1, 2, 2, 2), num_res_blocks=1, attn_resolutions=(16,),
                             resamp_with_conv=True, conditional=True, fir=True,
                             fir_kernel=[1, 3, 3, 1], skip_rescale=True, resblock_type="biggan",
                             progressive="none", progressive_input="residual",
                             progressive_combine="sum", attention_type="ddpm", init_scale=0.,
                             embedding_type="positional", fourier_scale=16, conv_size=3,
                             sigma_min=0.01, sigma_max=50, num_scales=1000, beta_min=0.1,
                             beta_max=20., dropout=0.0)
        c.optim = ConfigDict(weight_decay=0, optimizer="Adam", lr=2e-4, beta1=0.9, eps=1e-8,
                             warmup=5000, grad_clip=1.)
        c.device = torch.device("cpu")
        return c

    variants = {}
    c = base_config()
    variants["ncsnpp_a"] = c  # cifar10_ncsnpp_continuous-style at 32^2 x 1, nf 16
    c = base_config()
    c.model.update(progressive="output_skip", progressive_input="input_skip",
                   progressive_combine="cat", embedding_type="fourier", nf=8, num_res_blocks=1,
                   ch_mult=(1, 2, 2), attn_resolutions=(8,))
    c.data.update(image_size=16, num_channels=2, centered=True)
    variants["ncsnpp_b"] = c
    c = base_config()
    # resblock 'ddpm' is unreachable in the reference: its non-FIR Upsample passes 'nearest' as
    # scale_factor (layerspp.py:117) and its FIR path hits the negative-step slice
    # (up_or_down_sampling.py:126).  Variant c covers BigGAN blocks with naive resampling.
    c.model.update(resblock_type="biggan", fir=False, progressive_input="none", nf=8,
                   num_res_blocks=1, ch_mult=(1, 2), attn_resolutions=(8,), skip_rescale=False)
    c.data.update(image_size=16, num_channels=1)
    variants["ncsnpp_c"] = c
    c = base_config()
    c.model.update(name="ddpm", nf=32, ch_mult=(1, 1), num_res_blocks=1, attn_resolutions=(8,))
    c.data.update(image_size=16, num_channels=1)
    c.training.continuous = False
    c.sampling.update(predictor="ancestral_sampling", corrector="none")
    variants["ddpm_a"] = c

    def state_arrays(model):
        return {"p:" + k: v.detach().numpy() for k, v in model.state_dict().items()}

    nets = {}
    for name, cfg in variants.items():
        torch.manual_seed(0)
        model = mutils.get_model(cfg.model.name)(cfg)
        # the reference zero-inits Conv_1 / NIN_3 (init_scale 0); perturb every parameter so
        # that every path contributes to the output
        with torch.no_grad():
            for p in model.parameters():
                if p.requires_grad:
                    p.add_(torch.randn_like(p) * 0.02)
        model.eval()
        B = 3
        x = torch.rand(B, cfg.data.num_channels, cfg.data.image_size, cfg.data.image_size)
        if cfg.training.continuous:
            labels = torch.tensor([0.5, 999 * 0.37, 999.0])[:B] if cfg.model.embedding_type == \
                "positional" else torch.tensor([0.02, 1.5, 40.0])[:B]
        else:
            labels = torch.tensor([0, 37, 999])[:B]
        with torch.no_grad():
            y = model(x, labels)
        arr = state_arrays(model)
        arr.update(x=x.numpy(), labels=labels.numpy(), y=y.numpy(),
                   config_json=np.array(_config_json(cfg)))
        _save(f"net_{name}.npz", **arr)
        nets[name] = (cfg, model)

    # ------------------------------------------------------------- PC samplers
    def get_sde(cfg, N):
        # restatement of run_lib._get_sde (run_lib.py:45-58)
        if cfg.training.sde == "vpsde":
            return sde_lib.VPSDE(beta_min=cfg.model.beta_min, beta_max=cfg.model.beta_max, N=N), 1e-3
        raise NotImplementedError

    def record_pc(name, cfg, model, predictor, corrector, N, B, snr, n_steps, continuous):
        sde, eps = get_sde(cfg, N)
        shape = (B, cfg.data.num_channels, cfg.data.image_size, cfg.data.image_size)
        draws = []
        real = torch.randn_like

        def rec(t, *a, **k):
            z = real(t, *a, **k)
            draws.append(z.clone())
            return z

        torch.manual_seed(7)
        torch.randn_like = rec
        try:
            fn = sampling.get_pc_sampler(sde, shape, sampling.get_predictor(predictor),
                                         sampling.get_corrector(corrector), lambda v: v, snr,
                                         n_steps=n_steps, probability_flow=False,
                                         continuous=continuous, denoise=True, eps=eps,
                                         device="cpu")
            torch.manual_seed(11)
            prior = sde.prior_sampling(shape)
            torch.manual_seed(11)
            out, nfe = fn(model)
        finally:
            torch.randn_like = real
        arr = {"prior": prior.numpy(), "out": out.numpy(), "nfe": np.array(nfe),
               "draws": torch.stack(draws).numpy(), "N": np.array(N), "snr": np.array(snr),
               "n_steps": np.array(n_steps), "continuous": np.array(continuous),
               "predictor": np.array(predictor), "corrector": np.array(corrector),
               "net": np.array(net_of[name])}
        _save(f"pc_{name}.npz", **arr)

    net_of = {"em_langevin": "ncsnpp_a", "rd_ald": "ncsnpp_c", "anc_none": "ddpm_a",
              "em_none": "ncsnpp_b"}
    # N = 25: the smallest grids keep every DDPM beta = beta_max / N below 1 (N = 3 gives
    # sqrt(1 - beta) = NaN in the reference itself)
    record_pc("em_langevin", *nets["ncsnpp_a"], "euler_maruyama", "langevin", 25, 2, 0.075, 1, True)
    record_pc("rd_ald", *nets["ncsnpp_c"], "reverse_diffusion", "ald", 25, 2, 0.16, 2, True)
    record_pc("anc_none", *nets["ddpm_a"], "ancestral_sampling", "none", 25, 2, 0.16, 1, False)
    record_pc("em_none", *nets["ncsnpp_b"], "euler_maruyama", "none", 25, 2, 0.16, 1, True)

    # ------------------------------------------------------------- train steps
    def record_train(name, cfg, model, continuous, step0):
        model = mutils.get_model(cfg.model.name)(cfg)
        model.load_state_dict(nets[net_of_train[name]][1].state_dict())
        sde = sde_lib.VPSDE(beta_min=cfg.model.beta_min, beta_max=cfg.model.beta_max,
                            N=cfg.model.num_scales)
        opt = losses.get_optimizer(cfg, model.parameters())
        em = ema.ExponentialMovingAverage(model.parameters(), decay=cfg.model.ema_rate)
        state = dict(optimizer=opt, model=model, ema=em, step=step0)
        opt_fn = losses.optimization_manager(cfg)
        step_fn = losses.get_step_fn(sde, train=True, optimize_fn=opt_fn,
                                     reduce_mean=cfg.training.reduce_mean, continuous=continuous,
                                     likelihood_weighting=False)
        B = 4
        batch = torch.rand(B, cfg.data.num_channels, cfg.data.image_size, cfg.data.image_size)
        rand_log = []
        real_rand, real_randn_like, real_randint = torch.rand, torch.randn_like, torch.randint

        def rec_rand(*a, **k):
            v = real_rand(*a, **k)
            rand_log.append(("rand", v.clone()))
            return v

        def rec_randn_like(*a, **k):
            v = real_randn_like(*a, **k)
            rand_log.append(("randn_like", v.clone()))
            return v

        def rec_randint(*a, **k):
            v = real_randint(*a, **k)
            rand_log.append(("randint", v.clone()))
            return v

        params0 = {k: v.detach().clone() for k, v in model.named_parameters()}
        grads = {}
        real_step = opt.step

        def capture_then_step(*a, **k):
            for kk, p in model.named_parameters():
                if p.grad is not None:
                    grads[kk] = p.grad.detach().clone()
            return real_step(*a, **k)

        opt.step = capture_then_step
        torch.manual_seed(5)
        torch.rand, torch.randn_like, torch.randint = rec_rand, rec_randn_like, rec_randint
        try:
            loss = step_fn(state, batch)
        finally:
            torch.rand, torch.randn_like, torch.randint = real_rand, real_randn_like, real_randint
        arr = {"batch": batch.numpy(), "loss": np.array(loss.item(), np.float64),
               "step0": np.array(step0), "continuous": np.array(continuous),
               "net": np.array(net_of_train[name])}
        for i, (kind, v) in enumerate(rand_log):
            arr[f"rng{i}_{kind}"] = v.numpy()
        # initial parameters = the net_<name>.npz weights (not stored twice)
        for k, v in grads.items():
            arr["g:" + k] = v.numpy()
        for k, v in model.named_parameters():
            arr["p1:" + k] = v.detach().numpy()
        names = [k for k, p in model.named_parameters() if p.requires_grad]
        for k, s in zip(names, em.shadow_params):
            arr["ema:" + k] = s.numpy()
        _save(f"train_{name}.npz", **arr)

    net_of_train = {"dsm_ncsnpp": "ncsnpp_c", "dsm_fourier": "ncsnpp_b",
                    "ddpm_discrete": "ddpm_a"}
    record_train("dsm_ncsnpp", *nets["ncsnpp_c"], True, 2500)
    record_train("dsm_fourier", *nets["ncsnpp_b"], True, 0)
    record_train("ddpm_discrete", *nets["ddpm_a"], False, 2500)

    # ------------------------------------------------------------- fused leaky relu (CPU branch)
    x = torch.tensor(rng.standard_normal((3, 5, 4, 4)).astype(np.float32))
    b = torch.tensor(rng.standard_normal(5).astype(np.float32))
    y = fused_act.fused_leaky_relu(x, b, negative_slope=0.2, scale=2 ** 0.5)
    _save("fused_lrelu.npz", x=x.numpy(), b=b.numpy(), y=y.numpy())


if __name__ == "__main__":
    main()
