"""Benchmark: PC-sampler score-net evals/s (+ DSM train steps/s), NCSN++ 128x128x1.

BASELINE.json metric "PC-sampler score-net evals/s + train steps/s, NCSN++ 128^2 @1/2/4/8
MI355X", workload configs[2] (SURVEY.md 8d cfg #3): NCSN++ hyper-parameters of
configs/vp/cifar10_ncsnpp_continuous.py at 128x128x1, continuous VP-SDE N = 1000,
Euler-Maruyama predictor + Langevin corrector (snr 0.075, 1 corrector step), batch 64 per
GPU (weak scaling).  A "step" = one PC step over the batch = 2 score-net evaluations per
sample (corrector + predictor), fused update kernels, the whole step replayed from a
hipGraph.  Synthetic data: prior noise + random-init weights (no checkpoints offline).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  value = score-net evals/s of the whole job.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
# MIOpen compiles the backward-convolution kernels (DSM / PINN training, DPS input
# gradients) on first use; an in-tree cache directory (filled by an earlier run on the same
# image) skips minutes of compilation on a fresh box.  Set before torch loads MIOpen.
_MIOPEN_CACHE = os.path.join(REPO, "b-pinn-kalman-filter_amd", "miopen_cache")
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(_MIOPEN_CACHE, "kernels"))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(_MIOPEN_CACHE, "db"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

NCSNPP_GFLOP_PER_EVAL = 333.25     # SURVEY.md 8(d), FlopCounterMode, fwd, 128x128x1
NCSNPP_GFLOP_PER_TRAIN_SAMPLE = 999.10
FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md (f32-input MFMA = f32 vector peak)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="per-GPU batch (weak scaling)")
    ap.add_argument("--train-steps", type=int, default=6)
    ap.add_argument("--train-warmup", type=int, default=2)
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--cifar-steps", type=int, default=6,
                    help="configs[1] train steps (NCSN++ CIFAR-10 32x32x3, batch 128/GPU); 0: skip")
    ap.add_argument("--pinn-steps", type=int, default=10)
    ap.add_argument("--pinn-warmup", type=int, default=2)
    ap.add_argument("--pinn-graph", action="store_true",
                    help="replay the PINN forward/backward from a hipGraph (measured slower than "
                         "eager on ROCm 7: 3.66 vs 4.06 steps/s; needs --pinn-warmup >= 3)")
    ap.add_argument("--no-pinn", action="store_true")
    ap.add_argument("--dps-steps", type=int, default=2, help="accepted RK45 steps timed")
    ap.add_argument("--no-dps", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-samples", type=int, default=8,
                    help="CPU-baseline sample: 1 PC step on this many samples (~10 s on 16 cores)")
    ap.add_argument("--miopen-find", type=int, default=0,
                    help="1: MIOpen exhaustive find (cudnn.benchmark); immediate mode (0) picks "
                         "the same fp32 Winograd kernels for the forward and avoids minutes of "
                         "backward-conv searches")
    return ap.parse_args()


def build_model(dev, seed=0):
    import models  # noqa: F401
    from configs.vp import nc_ncsnpp_128
    from models import utils as mutils
    c = nc_ncsnpp_128.get_config()
    c.device = dev
    torch.manual_seed(seed)
    model = mutils.create_model(c, wrap=False)
    with torch.no_grad():  # random init everywhere (Conv_1 / NIN_3 are zero-init)
        for p in model.parameters():
            p.add_(torch.randn_like(p) * 0.01)
    return c, model


def _pmc_traffic(kernel_key):
    """HBM bytes per launch of a roofline kernel, from the committed PMC passes
    (profiles/r01_pmc_traffic.json: FETCH_SIZE x2 + WRITE_SIZE, same kernel and shape)."""
    try:
        with open(os.path.join(REPO, "profiles", "r01_pmc_traffic.json")) as f:
            return json.load(f)[kernel_key]["traffic_bytes"]
    except (OSError, KeyError, ValueError):
        return None


def time_kernel(fn, stream, reps=10):
    """Average duration (s) of fn() measured with HIP events on `stream`."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        for _ in range(3):
            fn()
        s.record(stream)
        for _ in range(reps):
            fn()
        e.record(stream)
    e.synchronize()
    return s.elapsed_time(e) / 1e3 / reps


def conv_roofline(dev, batch):
    """Dominant kernel of the score net (~75 % of a PC step): the fused, software-pipelined
    Winograd F(2x2,3x3) MFMA conv3x3 (csrc/conv_winograd.hip wino_f23_pipe_kernel), measured
    on its most frequent shape, 128 -> 128 channels @ 128x128 (13 per forward, SURVEY 8(a)
    a11).  MFMA-bound.

    achieved = the kernel's algorithmic MFMA FLOPs per launch -- Winograd F(2,3) multiplies
    16 transformed values per 2x2 output tile per (cin, cout), i.e. 4/9 of the direct
    convolution's 2*B*Cin*Cout*9*H*W -- over the HIP-event launch time on the launch
    stream.  `direct_equivalent_tflops` restates the same time against the direct-conv FLOP
    count (what MIOpen's implicit GEMM executes), `miopen_*` times F.conv2d on the same data."""
    import torch.nn.functional as F
    from op.conv import conv3x3, filter_transform
    x = torch.randn(batch, 128, 128, 128, device=dev)
    w = torch.randn(128, 128, 3, 3, device=dev) * 0.02
    st = torch.cuda.Stream(dev)
    with torch.cuda.stream(st):
        filter_transform(w)
        t = time_kernel(lambda: conv3x3(x, w), st)
        tm = time_kernel(lambda: F.conv2d(x, w, padding=1), st)
    direct = 2.0 * batch * 128 * 128 * 9 * 128 * 128
    wino = direct * 4.0 / 9.0
    ach = wino / t / 1e12
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
            "traffic": _pmc_traffic("wino_f23_pipe_kernel conv3x3 128->128 @128x128 B=64")
            if batch == 64 else None,
            "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
            "kernel": "wino_f23_pipe_kernel conv3x3 128->128 @128x128 fp32 (hand-written, f32 MFMA)",
            "ms_per_launch": round(t * 1e3, 4), "flop_per_launch": wino,
            "direct_equivalent_tflops": round(direct / t / 1e12, 2),
            "miopen_ms_per_launch": round(tm * 1e3, 4),
            "miopen_tflops": round(direct / tm / 1e12, 2)}


def upfirdn_roofline(dev, batch):
    """HBM roofline of upfirdn2d on the NCSN++ down2 shape [B,128,128,128] -> [B,128,64,64]."""
    from op import upfirdn2d
    k = torch.tensor(np.outer([1, 3, 3, 1], [1, 3, 3, 1]) / 64.0, dtype=torch.float32, device=dev)
    x = torch.randn(batch, 128, 128, 128, device=dev)
    st = torch.cuda.Stream(dev)
    with torch.cuda.stream(st):
        t = time_kernel(lambda: upfirdn2d(x, k, down=2, pad=(1, 1)), st)
    nbytes = 4.0 * (x.numel() + x.numel() // 4)
    ach = nbytes / t / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": _pmc_traffic("upfirdn2d down2 k4 [64,128,128,128]") if batch == 64 else None,
            "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
            "kernel": "upfirdn2d down2 k4 [B,128,128,128]", "ms_per_launch": round(t * 1e3, 4),
            "bytes_per_launch": nbytes}


def cpu_baseline(n_samples):
    """The oracle (torch-CPU restatement of the reference path) on the host cores: one warm-up
    PC step on 1 sample, then 1 PC step (EM + Langevin = 2 evals/sample) on n_samples."""
    from configs.vp import nc_ncsnpp_128
    from oracle import nets_ref, score_sde_ref
    import models  # noqa: F401
    from models import utils as mutils
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    c = nc_ncsnpp_128.get_config()
    c.device = "cpu"
    torch.manual_seed(0)
    params = nets_ref.init_params(mutils.create_model(c, wrap=False).state_dict())
    sde = score_sde_ref.SDESpec("vp", N=1000)
    mf = lambda x, t: nets_ref.forward(params, c, x, t)
    score_sde_ref.pc_sample(mf, sde, torch.randn(1, 1, 128, 128), "euler_maruyama", "langevin",
                            0.075, 1, True, n_iters=1)
    t0 = time.perf_counter()
    score_sde_ref.pc_sample(mf, sde, torch.randn(n_samples, 1, 128, 128), "euler_maruyama",
                            "langevin", 0.075, 1, True, n_iters=1)
    dt = time.perf_counter() - t0
    return {"value": round(2 * n_samples / dt, 4), "unit": "score-net evals/s", "cores": cores,
            "kind": "port",
            "sample": f"oracle/nets_ref + score_sde_ref: 1 PC step (EM+Langevin) on {n_samples} "
                      f"samples of 128x128x1, {dt:.1f}s, cpu={platform.processor() or 'x86_64'}"}


def pinn_batch(c, B, dev, seed=0):
    """Synthetic configs[3] batch (SURVEY.md 8d cfg #4): frames f1, f2 ~ U[0,1), coordinate
    channels = jittered meshes (an exact mesh puts sqrt(0) at the pixel holding both x.max()
    and y.max() and makes every x/y sensitivity NaN, in the reference too), t ~ U{300..899},
    target (u, v, p) ~ N(0, 0.25)."""
    g = torch.Generator(device=dev).manual_seed(seed)
    n = c.data.image_size
    lin = torch.linspace(0.05, 1.0, n, device=dev)
    f1 = torch.rand(B, 1, n, n, device=dev, generator=g)
    f2 = torch.rand(B, 1, n, n, device=dev, generator=g)
    x = (lin.view(1, 1, 1, n) + 0.01 * torch.rand(B, 1, n, n, device=dev, generator=g))
    y = (lin.view(1, 1, n, 1) + 0.01 * torch.rand(B, 1, n, n, device=dev, generator=g))
    t = torch.randint(300, 900, (B,), device=dev, generator=g).float()
    target = torch.randn(B, 3, n, n, device=dev, generator=g) * 0.5
    return (f1, f2, x.contiguous().requires_grad_(), y.contiguous().requires_grad_(),
            t.requires_grad_(), target)


def bench_cifar_train(args, ctx, dev):
    """configs[1]: NCSN++ continuous VP-SDE CIFAR-10 training (configs/vp/
    cifar10_ncsnpp_continuous.py: 32x32x3, nf 128, ch_mult (1,2,2,2), 4 res blocks, attention
    at 16^2), batch 128/GPU, synthetic data; DDP (RCCL gradient all-reduce) for N > 1."""
    import losses
    import models  # noqa: F401
    import sde_lib
    from configs.vp import cifar10_ncsnpp_continuous
    from models import utils as mutils
    from models.ema import ExponentialMovingAverage
    c = cifar10_ncsnpp_continuous.get_config()
    c.device = dev
    c.model.dropout = 0.0
    torch.manual_seed(0)
    model = mutils.create_model(c, wrap=False).train()
    tmodel = model
    if ctx.world_size > 1:
        tmodel = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index],
                                                           bucket_cap_mb=100)
    sde = sde_lib.VPSDE(c.model.beta_min, c.model.beta_max, c.model.num_scales)
    opt = losses.get_optimizer(c, tmodel.parameters())
    ema = ExponentialMovingAverage(tmodel.parameters(), decay=c.model.ema_rate)
    state = dict(optimizer=opt, model=tmodel, ema=ema, step=0)
    step_fn = losses.get_step_fn(sde, train=True, optimize_fn=losses.optimization_manager(c),
                                 reduce_mean=True, continuous=True)
    B = c.training.batch_size
    batch = torch.rand(B, 3, 32, 32, device=dev, generator=torch.Generator(device=dev).manual_seed(ctx.rank))
    for _ in range(2):
        step_fn(state, batch)
    torch.cuda.synchronize(dev)
    ctx.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.cifar_steps):
        loss = step_fn(state, batch)
    torch.cuda.synchronize(dev)
    ctx.barrier()
    torch.cuda.synchronize(dev)
    dt = ctx.all_reduce_max(time.perf_counter() - t0, dev)
    return {"cifar_train_steps_per_s": round(args.cifar_steps / dt, 3),
            "cifar_train_ms_per_step": round(dt / args.cifar_steps * 1e3, 2),
            "cifar_train_global_batch": B * ctx.world_size,
            "cifar_train_loss": round(float(loss.item()), 5),
            "cifar_config": "configs[1]: cifar10_ncsnpp_continuous 32x32x3, batch 128/GPU"}


def bench_pinn(args, ctx, dev):
    """configs[3]: one PINN train step (get_pinn_step_fn: FlowNet + PressureNet forward,
    equation_mse with create_graph first derivatives and second derivatives -- correlation and
    grid_sample grad2 on HIP --, backward, two Adams, EMA) at pinn_pde, batch 64/GPU, 64x64;
    gradients averaged over ranks with one coalesced RCCL all-reduce.  --pinn-graph replays the
    forward/backward from a hipGraph after two eager steps (opt-in: slower here)."""
    import losses
    from configs.pinn import pinn_pde
    from inverse.operators import get_operator
    from models.ema import ExponentialMovingAverage
    from pinn_kalman.pinn import PINN
    c = pinn_pde.get_config()
    c.device = dev
    torch.manual_seed(0)
    model = PINN(c)
    ema = ExponentialMovingAverage(model.parameters(), decay=c.model.ema_rate)
    opt_f = losses.get_optimizer(c, model.flownet.parameters())
    opt_p = losses.get_optimizer(c, model.pressurenet.parameters(), 0.005)
    state = dict(optimizer=(opt_f, opt_p), model=model, ema=ema, step=c.training.n_iters)
    step_fn = losses.get_pinn_step_fn(c, train=True, optimize_fn=losses.optimization_manager(c),
                                      ctx=ctx, graph=args.pinn_graph)
    operator = get_operator(c)
    batch = pinn_batch(c, args.batch, dev, seed=ctx.rank)
    for _ in range(args.pinn_warmup):
        step_fn(state, operator, batch)
    torch.cuda.synchronize(dev)
    ctx.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.pinn_steps):
        loss, pinn_loss, data_loss = step_fn(state, operator, batch)
    torch.cuda.synchronize(dev)
    ctx.barrier()
    torch.cuda.synchronize(dev)
    dt = ctx.all_reduce_max(time.perf_counter() - t0, dev)
    return {"pinn_train_steps_per_s": round(args.pinn_steps / dt, 3),
            "pinn_ms_per_step": round(dt / args.pinn_steps * 1e3, 2),
            "pinn_global_batch": args.batch * ctx.world_size,
            "pinn_losses": [round(float(v.item()), 6) for v in (loss, pinn_loss, data_loss)],
            "pinn_config": "configs[3]: pinn_pde (FlowNet 2.49M + PressureNet 7.54M), 64x64"}


def bench_dps(args, ctx, dev):
    """configs[4]: DPS conditional sampling (nc_ddpmpp_inpaint_dps at 256x256, DDPM++ 'ddpm'
    net, B = 16/GPU, inpainting with a Bernoulli(0.5) mask, variance 0.1, RK45 rtol = atol =
    1e-3).  Unit of work = one function evaluation (score forward + input gradient through
    the net) of the whole batch; timed over the first `--dps-steps` accepted RK45 steps
    (incl. the initial-step selection and any rejected attempts)."""
    import models  # noqa: F401
    from configs._configdict import ConfigDict
    from configs.vp import nc_ddpmpp
    from inverse.conditional_sampling import get_dps_sampler, get_solver
    from inverse.inverse_lib import get_obsvsde
    from inverse.operators import InpaintOperator
    from models import utils as mutils
    c = nc_ddpmpp.get_config()
    c.data.image_size = 256
    c.training.batch_size = 16
    c.device = dev
    c.inverse = ConfigDict(dict(operator="inpaint", invert=False, ratio=0.5, sampler="dps",
                                variance=0.1, solver="RK45", max_steps=args.dps_steps))
    torch.manual_seed(0)
    model = mutils.create_model(c, wrap=False).eval()
    with torch.no_grad():
        for p in model.parameters():
            p.add_(torch.randn_like(p) * 0.01)
    B, n = c.training.batch_size, 256
    g = torch.Generator(device=dev).manual_seed(1 + ctx.rank)
    mask = (torch.rand(1, 1, n, n, device=dev, generator=g) > 0.5).float().expand(B, 1, n, n)
    op = InpaintOperator(mask=[mask.contiguous()])
    origin = torch.rand(B, 1, n, n, device=dev, generator=g)
    obs, eps = get_obsvsde(c, op(origin, keep_shape=False), op)
    sampler = get_dps_sampler(c, obs, (B, 1, n, n), eps=eps, ctx=ctx if ctx.enabled else None)
    z = torch.randn(B, 1, n, n, device=dev, generator=g)
    c.inverse.max_steps = 1
    sampler(model, z=z)  # warm-up (kernel selection, allocator)
    c.inverse.max_steps = args.dps_steps
    torch.cuda.synchronize(dev)
    ctx.barrier()
    t0 = time.perf_counter()
    x = sampler(model, z=z)
    torch.cuda.synchronize(dev)
    ctx.barrier()
    dt = ctx.all_reduce_max(time.perf_counter() - t0, dev)
    nfe = get_solver.last_nfe
    return {"dps_nfe_per_s": round(nfe / dt, 3), "dps_sample_nfe_per_s": round(nfe * B * ctx.world_size / dt, 2),
            "dps_nfe_timed": nfe, "dps_global_batch": B * ctx.world_size,
            "dps_finite": bool(torch.isfinite(x).all().item()),
            "dps_config": "configs[4]: nc_ddpmpp_inpaint_dps @256x256 (ddpm net), B=16/GPU, RK45"}


_PHASE = ["start"]


def log(msg):
    _PHASE[0] = msg
    print(f"[bench] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)


def _heartbeat(period=45.0):
    """A line on stderr every `period` s while a phase runs (first-use MIOpen kernel
    compilation can keep a phase silent for minutes on a fresh box)."""
    import threading

    def run():
        t0 = time.time()
        while True:
            time.sleep(period)
            print(f"[bench] {time.strftime('%H:%M:%S')} ... ({_PHASE[0]}; {time.time() - t0:.0f}s)",
                  file=sys.stderr, flush=True)
    threading.Thread(target=run, daemon=True).start()


def main():
    args = parse()
    _heartbeat()
    import dist
    import sampling
    import sde_lib
    ctx = dist.init_from_env()
    torch.backends.cudnn.benchmark = bool(args.miopen_find)
    # one rank per GPU; more ranks than devices only in a gloo rehearsal on one box
    dev = torch.device("cuda", ctx.local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    world = ctx.world_size
    B = args.batch
    c, model = build_model(dev)
    model.eval()

    # ---------------------------------------------------------------- PC sampler
    sde = sde_lib.VPSDE(c.model.beta_min, c.model.beta_max, c.model.num_scales)
    eng = sampling.PCEngine(sde, (B, 1, 128, 128), sampling.EulerMaruyamaPredictor,
                            sampling.LangevinCorrector, c.sampling.snr, c.sampling.n_steps_each,
                            continuous=True, device=dev, seed=1234 + ctx.rank * 0,
                            use_graph=not args.no_graph, dist_ctx=ctx if world > 1 else None)
    log(f"rank {ctx.rank}/{world}: model built, capturing PC step")
    eng.reset(model)
    eng.advance(args.warmup)
    log("warm-up done, timing PC steps")
    torch.cuda.synchronize(dev)
    ctx.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    eng.advance(args.steps)
    torch.cuda.synchronize(dev)
    ctx.barrier()
    torch.cuda.synchronize(dev)
    dt = ctx.all_reduce_max(time.perf_counter() - t0, dev)
    x = eng._xm
    finite = bool(torch.isfinite(x).all().item())
    evals = 2 * B * world * args.steps  # (1 corrector + 1 predictor) score evals per sample/step
    evals_per_s = evals / dt
    ms_per_step = dt / args.steps * 1e3

    # ---------------------------------------------------------------- DSM train step
    train = None
    if not args.no_train:
        import losses
        from models.ema import ExponentialMovingAverage
        c.model.dropout = 0.0
        tmodel = model
        tmodel.train()
        if world > 1:
            tmodel = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index],
                                                               bucket_cap_mb=100)
        opt = losses.get_optimizer(c, tmodel.parameters())
        ema = ExponentialMovingAverage(tmodel.parameters(), decay=c.model.ema_rate)
        state = dict(optimizer=opt, model=tmodel, ema=ema, step=0)
        step_fn = losses.get_step_fn(sde, train=True, optimize_fn=losses.optimization_manager(c),
                                     reduce_mean=True, continuous=True)
        batch = torch.rand(B, 1, 128, 128, device=dev)
        log(f"sampler {evals_per_s:.1f} evals/s; train warm-up")
        for _ in range(args.train_warmup):
            step_fn(state, batch)
        torch.cuda.synchronize(dev)
        ctx.barrier()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(args.train_steps):
            loss = step_fn(state, batch)
        torch.cuda.synchronize(dev)
        ctx.barrier()
        torch.cuda.synchronize(dev)
        tdt = ctx.all_reduce_max(time.perf_counter() - t1, dev)
        train = {"train_steps_per_s": round(args.train_steps / tdt, 4),
                 "train_ms_per_step": round(tdt / args.train_steps * 1e3, 2),
                 "train_global_batch": B * world, "train_loss": round(float(loss.item()), 5),
                 "train_tflops": round(args.train_steps * B * world * NCSNPP_GFLOP_PER_TRAIN_SAMPLE
                                       / tdt / 1e3, 2)}

    cifar = None
    if args.cifar_steps > 0 and not args.no_train:
        log("configs[1] train steps (CIFAR-10 32x32, batch 128)")
        cifar = bench_cifar_train(args, ctx, dev)

    pinn = None
    if not args.no_pinn:
        log("PINN train steps")
        pinn = bench_pinn(args, ctx, dev)

    dps = None
    if not args.no_dps:
        log("DPS function evaluations")
        dps = bench_dps(args, ctx, dev)

    result = None
    if ctx.rank == 0:
        log("rooflines")
        roof = conv_roofline(dev, B)
        up_roof = upfirdn_roofline(dev, B)
        model_tflops = evals_per_s * NCSNPP_GFLOP_PER_EVAL / 1e3
        result = {
            "metric": "PC-sampler score-net evals/s (NCSN++ 128x128x1, EM + Langevin)",
            "value": round(evals_per_s, 3), "unit": "score-net evals/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (prior noise, random-init weights)",
            "config": {"workload": "configs[2]: NCSN++ 128x128x1 PC sampler, VP-SDE N=1000, "
                                   "euler_maruyama + langevin (snr 0.075), batch 64/GPU",
                       "model": "ncsnpp (62.69M params)", "global_batch": B * world,
                       "seq_len": None, "parallelism": f"dp{world} (batch-sharded, RCCL)",
                       "hip_graph": eng.graph is not None},
            "score_net_tflops": round(model_tflops, 2),
            "score_net_mfma_frac": round(model_tflops / FP32_MFMA_PEAK_TFLOPS, 4),
            "samples_finite": finite,
            "roofline": roof,
            "roofline_upfirdn2d": up_roof,
        }
        if train:
            result.update(train)
        if cifar:
            result.update(cifar)
        if pinn:
            result.update(pinn)
        if dps:
            result.update(dps)
    if world == 1 and not args.no_cpu_baseline and ctx.rank == 0:
        log("cpu baseline")
        result["cpu_baseline"] = cpu_baseline(args.cpu_samples)
        result["speedup_vs_cpu"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
    if ctx.rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
