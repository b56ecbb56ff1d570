"""GPU: the batch-sharded sampler and the DDP train step, 2 ranks on one device.

RCCL cannot put two ranks on one GPU, so these tests use the gloo backend with HIP
tensors; the code path (DistContext.all_reduce_sum_ between the captured graph segments,
DistributedDataParallel gradient averaging) is the one bench.py runs over RCCL."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import net_fixture, product_config

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _setup(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    sys.path[:0] = [HERE, os.path.join(HERE, "..", "b-pinn-kalman-filter_amd"),
                    os.path.join(HERE, "..")]
    import dist
    torch.cuda.set_device(0)
    return dist.init_from_env(backend="gloo")


def _model(dev):
    import models  # noqa: F401
    from models import utils as mutils
    cfg, sd, *_ = net_fixture("ncsnpp_a")
    c = product_config(cfg, dev)
    m = mutils.create_model(c, wrap=False)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return c, m


def _sampler_worker(rank, world, port, graph, q):
    try:
        ctx = _setup(rank, world, port)
        import sampling
        import sde_lib
        dev = torch.device("cuda:0")
        c, model = _model(dev)
        model.eval()
        torch.manual_seed(0)
        prior = torch.randn(4, 1, 32, 32)
        B = 4 // world
        sde = sde_lib.VPSDE(0.1, 20., 25)
        eng = sampling.PCEngine(sde, (B, 1, 32, 32), sampling.EulerMaruyamaPredictor,
                                sampling.LangevinCorrector, 0.075, 1, continuous=True, device=dev,
                                seed=77, use_graph=graph, dist_ctx=ctx)
        x, xm = eng.run(model, prior[rank * B:(rank + 1) * B], n_iters=6)
        q.put((rank, xm.cpu().numpy(), None))
        torch.distributed.destroy_process_group()
    except Exception as e:  # pragma: no cover - report to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29000 + (os.getpid() * 7 + world) % 2000
    ps = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=600) for _ in ps), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=120)
    for r in res:
        assert r[2] is None, r[2]
    return res


@pytest.mark.parametrize("graph", [True, False])
def test_batch_sharded_pc_sampler_matches_single_rank(graph):
    one = _run(_sampler_worker, 1, graph)[0][1]
    two = _run(_sampler_worker, 2, graph)
    both = np.concatenate([two[0][1], two[1][1]], 0)
    scale = max(1.0, float(np.abs(one).max()))
    # identical noise (Philox keyed by global sample index); only the float summation order
    # of the all-reduced batch-mean norms differs
    assert float(np.abs(both - one).max()) <= 1e-5 * scale


def _train_worker(rank, world, port, q):
    try:
        ctx = _setup(rank, world, port)
        import losses
        import sde_lib
        from models.ema import ExponentialMovingAverage
        dev = torch.device("cuda:0")
        c, model = _model(dev)
        model.train()
        if world > 1:
            model = torch.nn.parallel.DistributedDataParallel(model)
        g = torch.Generator().manual_seed(3)
        batch = torch.rand(4, 1, 32, 32, generator=g)
        t = torch.rand(4, generator=g) * (1 - 1e-5) + 1e-5
        z = torch.randn(4, 1, 32, 32, generator=g)
        B = 4 // world
        sl = slice(rank * B, (rank + 1) * B)
        draws = iter([t[sl].to(dev), z[sl].to(dev)])
        real_rand, real_randn_like = torch.rand, torch.randn_like
        torch.rand = lambda *a, **k: next(draws)
        torch.randn_like = lambda *a, **k: next(draws)
        sde = sde_lib.VPSDE(0.1, 20., 1000)
        opt = losses.get_optimizer(c, model.parameters())
        state = dict(optimizer=opt, model=model, step=1000,
                     ema=ExponentialMovingAverage(model.parameters(), 0.999))
        step_fn = losses.get_step_fn(sde, True, losses.optimization_manager(c), reduce_mean=True,
                                     continuous=True)
        step_fn(state, batch[sl].to(dev))
        torch.rand, torch.randn_like = real_rand, real_randn_like
        flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy()
        q.put((rank, flat, None))
        if world > 1:
            torch.distributed.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, None, traceback.format_exc()))


def test_ddp_train_step_matches_single_rank():
    one = _run(_train_worker, 1)[0][1]
    two = _run(_train_worker, 2)
    np.testing.assert_allclose(two[0][1], two[1][1], rtol=0, atol=0)  # replicas stay identical
    # Adam's first step moves every parameter by ~lr * sign(grad) (lr = 2e-4 * 1000/5000 warm-up):
    # a gradient within rounding of zero may flip sign between the sharded and the full-batch
    # reduction order, so allow one Adam step of difference
    diff = np.abs(two[0][1] - one)
    assert diff.max() <= 2 * 4e-5 + 1e-6
    assert (diff > 1e-5).mean() < 1e-4


def _sim_worker(rank, world, port, compat, q):
    try:
        ctx = _setup(rank, world, port)
        from pinn_kalman import simulator
        rng = np.random.default_rng(0)
        begin = np.zeros((2, 6, 200, 200), np.float32)
        begin[:, 2] = rng.uniform(0.1, 1.0, (2, 200, 200))
        begin[:, 3:5] = rng.uniform(0.05, 0.5, (2, 2, 200, 200)) * rng.choice([-1, 1], (2, 2, 200, 200))
        begin[:, 5] = rng.normal(0, 0.01, (2, 200, 200))
        res, vel, pres = simulator.step(None, begin, t_range=(0, 3), replicas=8,
                                        device=torch.device("cuda:0"), ctx=ctx, compat=compat)
        q.put((rank, [np.stack([r.cpu().numpy() for r in a]) for a in (res, vel, pres)], None))
        if world > 1:
            torch.distributed.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, None, traceback.format_exc()))


def test_sharded_simulator_equals_single_process_bit_for_bit():
    """pinn_kalman.simulator.step(ctx=...): rank r rolls replicas [4r, 4r + 4) of 8, no
    collective.  compat=False (independent replicas): the shards equal the single-process
    rollout exactly.  compat=True: the reference's unbind quirk couples sample b to velocity
    planes b, b + 1 (samples b / 2 ...), so a shard reproduces the reference run of its own
    R replicas -- the single-process rollout at replicas = R -- bit for bit."""
    one = _run(_sim_worker, 1, False)[0][1]
    two = _run(_sim_worker, 2, False)
    for k in range(3):
        both = np.concatenate([two[0][1][k], two[1][1][k]], 1)  # [steps, replicas, ...]
        np.testing.assert_array_equal(both, one[k])
    two_c = _run(_sim_worker, 2, True)
    eight = _run(_sim_worker, 1, True)[0][1]  # replicas=8 in one process
    for k in range(3):
        # sample b < 4 only ever reads planes of samples <= (b + 1) / 2 < 4: the first shard
        # equals the first four replicas of the 8-replica rollout, and both shards (same
        # initial replicas) are identical
        np.testing.assert_array_equal(two_c[0][1][k], eight[k][:, :4])
        np.testing.assert_array_equal(two_c[1][1][k], two_c[0][1][k])


def _pinn_worker(rank, world, port, nan_rank, q):
    try:
        ctx = _setup(rank, world, port)
        import losses
        from configs.pinn import pinn_pde
        from conftest import build_pinn_weights, load_golden, small_config
        from inverse.operators import InpaintOperator
        from models.ema import ExponentialMovingAverage
        from pinn_kalman.pinn import PINN
        dev = torch.device("cuda:0")
        c = small_config(pinn_pde.get_config)
        m = build_pinn_weights(PINN, c).to(dev)
        c.device = dev
        c.inverse.variance = 0.0  # the measurement noise draws then do not matter
        d = load_golden("pinn_step.npz")
        B = 2 // world
        sl = slice(rank * B, (rank + 1) * B)
        T = lambda k: torch.tensor(d[k][sl].copy(), device=dev)
        batch = [T("f1"), T("f2"), T("x").requires_grad_(), T("y").requires_grad_(),
                 T("t").requires_grad_(), T("target")]
        if rank == nan_rank:  # the pressure target: reaches PressureNet's last conv
            batch[5][0, 2, 3, 3] = float("nan")
        op = InpaintOperator(mask=[torch.tensor(d["mask"][sl].copy(), device=dev)])
        em = ExponentialMovingAverage(m.parameters(), decay=c.model.ema_rate)
        opt_f = losses.get_optimizer(c, m.flownet.parameters())
        opt_p = losses.get_optimizer(c, m.pressurenet.parameters(), 0.001)
        state = dict(optimizer=(opt_f, opt_p), model=m, ema=em, step=50)
        grads = {}
        for opt, pref in ((opt_f, "flownet."), (opt_p, "pressurenet.")):
            net = getattr(m, pref[:-1])

            def capture(*a, _real=opt.step, _net=net, _pref=pref, **k):
                for kk, p in _net.named_parameters():
                    if p.grad is not None:
                        grads[_pref + kk] = p.grad.detach().reshape(-1).cpu().numpy()
                return _real(*a, **k)

            opt.step = capture
        p0 = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
        step_fn = losses.get_pinn_step_fn(c, train=True, optimize_fn=losses.optimization_manager(c),
                                          ctx=ctx if world > 1 else None)
        losses_out = step_fn(state, op, tuple(batch))
        p1 = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
        g = np.concatenate([grads[k] for k in sorted(grads)]) if grads else None
        q.put((rank, (state["step"], g, p1, p0, [float(v) for v in losses_out]), None))
        if world > 1:
            torch.distributed.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, None, traceback.format_exc()))


def test_sharded_pinn_step_matches_single_rank():
    """get_pinn_step_fn(ctx=...) on 2 ranks x 1 sample == 1 rank x 2 samples: the
    bucketed, backward-overlapped gradient average equals the full-batch gradient (each
    rank's loss is the mean over its shard; fp32 reduction order differs)."""
    (_, (s1, g1, p1, _, l1), _), = _run(_pinn_worker, 1, -1)
    two = _run(_pinn_worker, 2, -1)
    (s_a, g_a, pa, _, la), (s_b, g_b, pb, _, lb) = two[0][1], two[1][1]
    assert s1 == s_a == s_b == 51
    np.testing.assert_array_equal(g_a, g_b)
    np.testing.assert_array_equal(pa, pb)  # replicas stay identical
    assert np.abs(g_a - g1).max() <= 2e-3 * np.abs(g1).max()
    np.testing.assert_allclose(0.5 * (la[0] + lb[0]), l1[0], rtol=2e-4)


def test_nan_on_one_rank_makes_every_rank_skip():
    """A NaN in rank 1's pressure target: its gradient reaches every rank through the all-reduce,
    so both ranks take the reference's NaN skip (losses.py:361-366) -- no optimizer step,
    no EMA update, step counter unchanged, parameters unchanged on both."""
    two = _run(_pinn_worker, 2, 1)
    for _, (step, g, p1, p0, _), _ in two:
        assert step == 50
        np.testing.assert_array_equal(p1, p0)


def _pinn_graph_worker(rank, world, port, q):
    """4 PINN train steps of the sharded graph step and of the sharded eager step (same model,
    batch shard and noise) on this rank; returns both runs' losses and final parameters."""
    try:
        ctx = _setup(rank, world, port)
        import copy

        import losses
        from configs.pinn import pinn_pde
        from conftest import build_pinn_weights, load_golden, small_config
        from inverse.operators import InpaintOperator
        from models.ema import ExponentialMovingAverage
        from op import conv as conv_op
        from pinn_kalman.pinn import PINN
        dev = torch.device("cuda:0")
        c = small_config(pinn_pde.get_config)
        m0 = build_pinn_weights(PINN, c).to(dev)
        c.device = dev
        d = load_golden("pinn_step.npz")
        B = 2 // world
        sl = slice(rank * B, (rank + 1) * B)
        T = lambda k: torch.tensor(d[k][sl].copy(), device=dev)
        out = {}
        for graph in (True, False):
            m = copy.deepcopy(m0)
            em = ExponentialMovingAverage(m.parameters(), decay=c.model.ema_rate)
            state = dict(optimizer=(losses.get_optimizer(c, m.flownet.parameters()),
                                    losses.get_optimizer(c, m.pressurenet.parameters(), 0.001)),
                         model=m, ema=em, step=50)
            op = InpaintOperator(mask=[torch.tensor(d["mask"][sl].copy(), device=dev)])
            step_fn = losses.get_pinn_step_fn(c, train=True, ctx=ctx, graph=graph,
                                              optimize_fn=losses.optimization_manager(c))
            ls = []
            torch.manual_seed(11 + rank)
            with conv_op.native_only():
                for _ in range(4):
                    batch = (T("f1"), T("f2"), T("x").requires_grad_(), T("y").requires_grad_(),
                             T("t").requires_grad_(), T("target"))
                    ls.append([float(v) for v in step_fn(state, op, batch)])
            out[graph] = (ls, torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy())
        q.put((rank, out, None))
        torch.distributed.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, None, traceback.format_exc()))


def test_sharded_pinn_graph_step_matches_sharded_eager_step():
    """get_pinn_step_fn(graph=True, ctx=...) on 2 ranks (the gradient all-reduce runs eagerly
    between the two graph replays of a step): losses of 4 steps and the final parameters ==
    the sharded eager step's on each rank, and the two ranks' replicas stay identical
    (the multi-rank graph path compared with the eager one)."""
    two = _run(_pinn_graph_worker, 2, )
    for _, out, _ in two:
        lg, pg = out[True]
        le, pe = out[False]
        lg, le = np.array(lg), np.array(le)
        np.testing.assert_allclose(lg[:, [0, 2]], le[:, [0, 2]], rtol=1e-5, atol=0)
        np.testing.assert_allclose(lg[:, 1], le[:, 1], rtol=2e-3, atol=1e-9)
        assert np.abs(pg - pe).max() <= 4e-3
    np.testing.assert_array_equal(two[0][1][True][1], two[1][1][True][1])


def _rccl_capture_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0",
                          WORLD_SIZE="1", LOCAL_RANK="0")
        import torch.distributed as tdist
        torch.cuda.set_device(0)
        tdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        t = torch.zeros(2, device="cuda:0")
        tdist.all_reduce(t)  # communicator up before the capture (as the PC warm-up does)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            t.add_(1.0)
            tdist.all_reduce(t)
        torch.cuda.current_stream().wait_stream(s)
        t.zero_()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            t.add_(1.0)
            tdist.all_reduce(t)
        t.zero_()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        q.put((0, t.cpu().numpy(), None))
        tdist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((0, None, traceback.format_exc()))


def test_rccl_all_reduce_captures_in_a_hip_graph():
    """The mechanics behind BPK_PC_GRAPH_ALLREDUCE=1 (sampling._graph_collective: the sharded
    PC step as one graph with the Langevin all-reduce inside): an RCCL all-reduce captured in
    a hipGraph replays (one rank: two ranks cannot share a device under RCCL)."""
    (r,) = _run(_rccl_capture_worker, 1)
    np.testing.assert_array_equal(r[1], np.full(2, 3.0, np.float32))


def test_bench_gpus_2_matches_world_1_samples():
    """`python bench.py --gpus 2` (gloo, both ranks on the one device) launches two ranks,
    shards the global batch (strong scaling, the configs[2] form: --global-batch 8 -> 4 per
    rank), reports n_gpus 2 and produces the samples of the single-rank run (Philox noise
    keyed by the global sample index; the Langevin batch-mean norm summed over ranks)."""
    import json
    import subprocess
    bench = os.path.join(HERE, "..", "bench.py")
    common = ["--steps", "3", "--warmup", "1", "--global-batch", "8", "--no-train", "--no-pinn",
              "--no-dps", "--ns-steps", "0", "--ncddpmpp-steps", "0", "--no-cpu-baseline",
              "--no-roofline", "--sample-sums"]
    out = {}
    for n in (1, 2):
        env = dict(os.environ, BPK_DIST_BACKEND="gloo")
        env.pop("WORLD_SIZE", None)
        p = subprocess.run([sys.executable, bench, "--gpus", str(n)] + common, env=env,
                           capture_output=True, text=True, timeout=400)
        assert p.returncode == 0, p.stderr[-3000:]
        out[n] = json.loads(p.stdout.strip().splitlines()[-1])
    assert out[1]["n_gpus"] == 1 and out[2]["n_gpus"] == 2
    assert out[2]["scaling"] == "strong"
    assert out[2]["config"]["global_batch"] == 8 and out[2]["config"]["per_gpu_batch"] == 4
    a, b = np.array(out[1]["sample_sums"]), np.array(out[2]["sample_sums"])
    assert a.shape == b.shape == (8,)
    np.testing.assert_allclose(b, a, rtol=1e-5, atol=1e-3 * np.abs(a).max())
