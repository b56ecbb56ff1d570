"""hipGraph replays with arbitrary eager work between them.

Round 4 found that eager reductions between replays of the captured PINN step corrupted later
replays.  The cause was the HIP runtime's graph packet capture, which leaves a graph's kernel
arguments in the eager launch ring (op/_hipenv.py); with the runtime setting in effect, these
tests interleave exactly that kind of work -- the reference loop's eval step
(pinn_lib.py:154-162), device reductions, ~1 MB of large-argument kernel launches, and a
caller's zero_grad(set_to_none=True) -- between graph steps and demand the eager results.
"""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _flood(dev):
    """eager launches carrying large kernel-argument blocks (non-contiguous elementwise ops and
    reductions): ~1.3 MB of arguments, enough to wrap the runtime's launch ring"""
    a = torch.randn(256, 512, device=dev)
    acc = torch.zeros((), device=dev)
    for _ in range(600):
        acc = acc + (a.t() + a.t()).abs().sum()
    return float(acc)


def test_hip_runtime_setting_in_effect():
    from op import _hipenv
    assert _hipenv.graph_replays_safe()


@pytest.mark.parametrize("B", [64, 8])
def test_pinn_graph_step_with_eval_steps_and_reductions_matches_eager_b64(hip, B):
    """The bench configuration (configs[3], B = 64; B = 8: a rank of the 8-GPU point, whose
    step batches the residual's derivative passes over input copies): 5 train steps as hipGraph replays with, after
    each, an eager eval step (get_pinn_step_fn(train=False): EMA store / copy_to / restore and a
    forward with the residual), device reductions of every gradient, a large-argument launch
    flood and zero_grad(set_to_none=True) -- vs the same loop with the eager train step: train
    and eval losses at every step and the final parameters, at the tolerances of
    test_pinn_step_hip_graph_replays_match_eager."""
    import losses
    from configs.pinn import pinn_pde
    from inverse.operators import InpaintOperator
    from models.ema import ExponentialMovingAverage
    from op import conv as conv_op
    from pinn_kalman.pinn import PINN
    c = pinn_pde.get_config()
    c.device = hip
    torch.manual_seed(0)
    m0 = PINN(c)
    n, steps = c.data.image_size, 5
    g = torch.Generator().manual_seed(2)
    lin = torch.linspace(0.05, 1.0, n)

    def batch():
        f1, f2 = torch.rand(B, 1, n, n, generator=g), torch.rand(B, 1, n, n, generator=g)
        x = lin.view(1, 1, 1, n) + 0.01 * torch.rand(B, 1, n, n, generator=g)
        y = lin.view(1, 1, n, 1) + 0.01 * torch.rand(B, 1, n, n, generator=g)
        t = torch.randint(300, 900, (B,), generator=g).float()
        target = torch.randn(B, 3, n, n, generator=g) * 0.5
        return [v.to(hip) for v in (f1, f2, x, y, t, target)]
    train_b = [batch() for _ in range(steps)]
    eval_b = [batch() for _ in range(steps)]
    masks = [(torch.rand(1, 1, n, n, generator=g) > 0.3).float().expand(B, 1, n, n).contiguous()
             for _ in range(3)]

    def run(graph):
        m = copy.deepcopy(m0).to(hip)
        ema = ExponentialMovingAverage(m.parameters(), decay=c.model.ema_rate)
        opts = (losses.get_optimizer(c, m.flownet.parameters()),
                losses.get_optimizer(c, m.pressurenet.parameters(), 0.005))
        state = dict(optimizer=opts, model=m, ema=ema, step=c.training.n_iters)
        train_fn = losses.get_pinn_step_fn(c, train=True, graph=graph,
                                           optimize_fn=losses.optimization_manager(c))
        eval_fn = losses.get_pinn_step_fn(c, train=False, optimize_fn=None)
        op = InpaintOperator(mask=masks)
        tr, ev, gsum = [], [], []
        torch.manual_seed(321)
        with conv_op.native_only():
            for bt, be in zip(train_b, eval_b):
                x, y, t = (v.clone().requires_grad_() for v in bt[2:5])
                tr.append([float(v.detach()) for v in train_fn(state, op, (bt[0], bt[1], x, y, t, bt[5]))])
                # the reference loop's eval step (pinn_lib.py:154-162) on the device between
                # train steps, then metrics-style reductions and a launch flood
                x, y, t = (v.clone().requires_grad_() for v in be[2:5])
                ev.append([float(v.detach()) for v in eval_fn(state, op, (be[0], be[1], x, y, t, be[5]))])
                gsum.append(float(sum(p.grad.double().abs().sum() for p in m.parameters()
                                      if p.grad is not None)))
                _flood(hip)
                for o in opts:
                    o.zero_grad(set_to_none=True)
        m.train()
        return np.array(tr), np.array(ev), np.array(gsum), [p.detach().clone() for p in m.parameters()]
    tg, eg, gg, pg = run(True)
    te, ee, ge, pe = run(False)
    np.testing.assert_allclose(tg[:, [0, 2]], te[:, [0, 2]], rtol=1e-5, atol=0)
    np.testing.assert_allclose(tg[:, 1], te[:, 1], rtol=2e-3, atol=0)
    np.testing.assert_allclose(eg[:, [0, 2]], ee[:, [0, 2]], rtol=1e-5, atol=0)
    np.testing.assert_allclose(eg[:, 1], ee[:, 1], rtol=2e-3, atol=0)
    np.testing.assert_allclose(gg, ge, rtol=1e-3, atol=0)  # the gradients the optimizers saw
    for a, b in zip(pg, pe):
        assert (a - b).abs().max().item() <= 4e-3


def test_pc_sampler_graph_with_eager_work_between_steps_is_bit_exact(hip):
    """The PC sampler's step graph (bench config, B = 8): 16 replays with a large-argument launch
    flood and reductions between every two steps give bit-identical samples to 16 replays
    without (same prior; the step noise is counter-based)."""
    import sampling
    import sde_lib
    from bench import build_model
    c, model = build_model(hip)
    model.eval()
    sde = sde_lib.VPSDE(c.model.beta_min, c.model.beta_max, c.model.num_scales)
    outs = []
    prior = torch.randn(8, 1, 128, 128, generator=torch.Generator().manual_seed(5))
    for work in (False, True):
        eng = sampling.PCEngine(sde, (8, 1, 128, 128), sampling.EulerMaruyamaPredictor,
                                sampling.LangevinCorrector, c.sampling.snr, 1, continuous=True,
                                device=hip, seed=1234)
        assert eng.use_graph
        eng.reset(model, x_init=prior)  # the same prior in both runs
        for _ in range(16):
            eng.advance(1)
            if work:
                _flood(hip)
        torch.cuda.synchronize()
        assert eng.graph is not None
        outs.append(eng._xm.clone())
        del eng
    assert torch.equal(outs[0], outs[1])
