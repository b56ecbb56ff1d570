"""Benchmark: PC-sampler score-net evals/s (+ DSM train steps/s), NCSN++ 128x128x1.

BASELINE.json metric "PC-sampler score-net evals/s + train steps/s, NCSN++ 128^2 @1/2/4/8
MI355X", workload configs[2] (SURVEY.md 8d cfg #3): NCSN++ hyper-parameters of
configs/vp/cifar10_ncsnpp_continuous.py at 128x128x1, continuous VP-SDE N = 1000,
Euler-Maruyama predictor + Langevin corrector (snr 0.075, 1 corrector step), global batch
64 sharded 64/N per GPU (strong scaling: BASELINE configs[2] "batch=64, 1->8 GPUs", SURVEY
8(e) "64 -> 8/GPU"; the reference's nn.DataParallel scatters one global batch,
models/utils.py:93).  A "step" = one PC step over the batch = 2 score-net evaluations per
sample (corrector + predictor), fused update kernels, the whole step replayed from a
hipGraph.  Synthetic data: prior noise + random-init weights (no checkpoints offline).
The other phases shard their own config's global batch the same way (DSM train 64, PINN 64,
DPS 16, nc_ddpmpp 64, CIFAR 128); the ns_step simulator runs independent replicas (256 per
GPU).  `--weak` (or an explicit per-GPU `--batch`) gives every rank the whole batch.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--global-batch 64] [--weak]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  value = score-net evals/s of the whole job.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
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
from op import _hipenv  # noqa: E402,F401  (HIP graph-replay setting, before torch)

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
    ap.add_argument("--global-batch", type=int, default=64,
                    help="configs[2] global batch, sharded global/N per GPU (strong scaling)")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling: every rank runs the whole global batch of every phase")
    ap.add_argument("--per-rank-of", type=int, default=None, metavar="N",
                    help="run every phase at the per-rank batch of an N-GPU strong-scaled run, "
                         "on this process's GPU(s) (--per-rank-of 8 on one GPU: the work of each "
                         "rank of the 8-GPU point); the line reports this process's rates")
    ap.add_argument("--batch", type=int, default=None,
                    help="explicit per-GPU batch of the sampler / DSM / PINN / nc_ddpmpp phases "
                         "(weak scaling; e.g. --batch 8 at N=1 is the per-rank work of N=8)")
    ap.add_argument("--train-steps", type=int, default=6)
    ap.add_argument("--train-warmup", type=int, default=2)
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--cifar-steps", type=int, default=6,
                    help="configs[1] train steps (NCSN++ CIFAR-10 32x32x3, batch 128/GPU); 0: skip")
    ap.add_argument("--pinn-steps", type=int, default=10)
    ap.add_argument("--pinn-warmup", type=int, default=2)
    ap.add_argument("--no-pinn", action="store_true")
    ap.add_argument("--pinn-eager", action="store_true",
                    help="time the eager PINN step instead of its hipGraph replay")
    ap.add_argument("--dps-steps", type=int, default=2, help="accepted RK45 steps timed")
    ap.add_argument("--no-dps", action="store_true")
    ap.add_argument("--ns-steps", type=int, default=20, help="ns_step full steps timed; 0: skip")
    ap.add_argument("--ncddpmpp-steps", type=int, default=10,
                    help="nc_ddpmpp (ddpm, ancestral) 128^2 PC steps timed; 0: skip")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-samples", type=int, default=8,
                    help="CPU-baseline sample: 1 PC step on this many samples (~10 s on 16 cores)")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--sample-sums", action="store_true",
                    help="add the per-sample sums of x_mean (global sample order) to the line")
    ap.add_argument("--plumbing", action="store_true",
                    help="launcher / rendezvous check only (no GPU work): each rank all-reduces "
                         "its rank id and rank 0 prints the line skeleton")
    ap.add_argument("--miopen-find", type=int, default=0,
                    help="1: MIOpen exhaustive find (cudnn.benchmark); immediate mode (0) picks "
                         "the same fp32 Winograd kernels for the forward and avoids minutes of "
                         "backward-conv searches")
    return ap.parse_args()


def shard(args, world, global_b, explicit=True):
    """Per-rank batch of a phase whose config fixes the global batch `global_b`: global/N
    (strong scaling), the whole batch per rank with --weak, or the explicit
    per-GPU --batch for the phases that take it."""
    if explicit and args.batch is not None:
        return args.batch
    if args.weak:
        return global_b
    if args.per_rank_of:
        world = world * args.per_rank_of
    if global_b % world:
        raise SystemExit(f"[bench] global batch {global_b} does not shard over {world} ranks")
    return global_b // world


def scaling_mode(args):
    return "weak" if (args.weak or args.batch is not None) else "strong"


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


def time_kernel_graph(fn, stream, reps=20):
    """Average duration (s) of fn() with `reps` launches captured in one hipGraph and timed
    with HIP events around its replays: short kernels (tens of us) are not stretched by the
    host's per-call overhead between eager launches."""
    with torch.cuda.stream(stream):
        for _ in range(3):
            fn()
    stream.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        for _ in range(reps):
            fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        g.replay()
        s.record(stream)
        for _ in range(3):
            g.replay()
        e.record(stream)
    e.synchronize()
    return s.elapsed_time(e) / 1e3 / (3 * reps)


# The sampler's dominant kernel: the Winograd conv with the GroupNorm+SiLU prologue
# (csrc/conv_winograd.hip wino_f23_k16_kernel<true>), ~77 % of a PC step.  Its roofline
# is taken over the NCSN++ 128x128 shape mix it runs in the sampler: per (cin, cout, hw) the
# PRE form with bias + GroupNorm partial statistics (Conv_0 of a BigGAN block) and with the
# residual tail (Conv_1), weighted by their counts per forward: the
# census of one forward of the bench model (tools/conv_census.py, profiles/r02_conv_census.txt;
# the up path's two-source convs are timed as one source of Cin = C1 + C2, same kernel and
# FLOPs).
WINO_MIX = [  # (cin, cout, hw, PRE+stats convs per forward, PRE+residual+stats convs per forward)
    (128, 128, 128, 4, 9), (256, 128, 128, 4, 0), (384, 128, 128, 1, 0), (256, 256, 128, 0, 1),
    (128, 128, 64, 0, 1), (128, 256, 64, 1, 0), (256, 256, 64, 3, 10), (384, 256, 64, 1, 0),
    (512, 256, 64, 4, 0), (256, 256, 32, 4, 11), (512, 256, 32, 5, 0), (256, 256, 16, 6, 12),
    (512, 256, 16, 5, 0)]


CSRC = os.path.join(REPO, "b-pinn-kalman-filter_amd", "csrc")
# the kernel sources each PMC entry's counted dispatches come from ("*": every source)
PMC_SOURCES = {"wino_pre_mix": ["conv_winograd.hip"], "upfirdn2d": ["upfirdn2d.hip"],
               "ns_step": ["ns_step.hip"], "step": ["*"]}


def src_sha1(names):
    """{file: sha1} of the listed csrc/ sources ("*": all of them), as tools/pmc_summary.py
    records them next to the counters it summarises."""
    import glob
    import hashlib
    files = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h"))) \
        if names == ["*"] else [os.path.join(CSRC, n) for n in names]
    return {os.path.basename(f): hashlib.sha1(open(f, "rb").read()).hexdigest() for f in files}


def _pmc_entry(key, section="traffic"):
    """The newest committed PMC entry for `key` (profiles/r0*_pmc_<section>.json) whose
    recorded kernel sources are the ones this tree builds; None when the entry was measured
    on other kernels (or carries no source record): counters of a kernel that no longer
    runs are never attached to a live measurement."""
    import glob
    want = next(v for k, v in PMC_SOURCES.items() if key.startswith(k))
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", f"r0*_pmc_{section}.json")),
                       reverse=True):
        try:
            with open(path) as f:
                e = json.load(f)[key]
        except (OSError, KeyError, ValueError):
            continue
        rec = e.get("src_sha1") if isinstance(e, dict) else None
        if rec is None or rec != src_sha1(want):
            return None
        return e, os.path.basename(path)
    return None


def _pmc(key):
    """HBM bytes of a roofline kernel (FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md
    gfx950 correction; tools/pmc_summary.py), or None when no PMC pass measured the kernels
    this tree runs."""
    got = _pmc_entry(key)
    return None if got is None else got[0]["traffic_bytes"]


def step_roofline(tally, steps_per_s, what, unit_of_work="step", survey_direct=None,
                  traffic_key=None):
    """Roofline object of a whole step (train / PINN / DPS rows): achieved =
    executed FLOPs of one counted step (op.flops: every native MFMA launch on its executed
    basis -- Winograd 4/9 of direct --, aten matmuls / MIOpen convs via FlopCounterMode on
    the direct basis) x steps/s, against the f32 MFMA peak."""
    ex, di = tally.total_executed, tally.total_direct
    ach = ex * steps_per_s / 1e12
    # traffic: HBM bytes of every kernel of one counted step / nfe (rocprofv3 FETCH_SIZE x 2 +
    # WRITE_SIZE between marker dispatches, tools/prof_steps.py + tools/pmc_summary.py)
    out = {"bound": "mfma", "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
           "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
           "traffic": _pmc(traffic_key) if traffic_key else None,
           "kernel": what, "flop_basis": "executed (native kernels as issued; aten ops direct)",
           f"executed_flop_per_{unit_of_work}": ex, f"direct_flop_per_{unit_of_work}": di,
           "direct_basis_tflops": round(di * steps_per_s / 1e12, 2),
           "native_flop_by_kind": {k: round(v["executed"] / 1e12, 4)
                                   for k, v in tally.summary()["native"].items()},
           "aten_flop": tally.aten}
    if survey_direct is not None:
        out["survey_direct_flop_per_" + unit_of_work] = survey_direct
    return out


def _phase_reset(dev):
    """Before a phase: the previous phases' tensors collected and the caching allocator's free
    blocks returned, so each phase allocates as it would in its own process (the CIFAR phase
    measured 12.8-13.6 steps/s after the sampler and DSM phases, 14.4-14.7 without them)."""
    import gc
    gc.collect()
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()


def counted(fn, dev):
    """fn() once inside an op.flops counting block (outside any timed region)."""
    from op import flops
    with flops.counting() as tally:
        r = fn()
    torch.cuda.synchronize(dev)
    return tally, r


def _ns_valu_cycles():
    """SIMD-cycles of VALU issue per ns_step full step at B=256, 192^2: SQ_ACTIVE_INST_VALU
    (quad-cycles) x 4 of the velocity launch + the pressure/density launch, from the committed
    PMC pass of the kernels this tree builds (profiles/r0*_pmc_sq.json, src_sha1 checked; the
    instruction stream does not depend on the data)."""
    got = _pmc_entry("ns_step launches (3 full steps)", "sq")
    if got is None:
        return None, None
    per = {}
    for r in got[0]["runs"]:
        per.setdefault(r["_grid"], []).append(4.0 * r["SQ_ACTIVE_INST_VALU"])
    return sum(sum(v) / len(v) for v in per.values()), got[1]


def wino_mix_times(dev, batch, reps=10):
    """Per-shape HIP-event launch times (s) of the PRE+stats and PRE+residual forms."""
    from op.conv import conv3x3, filter_transform
    st = torch.cuda.Stream(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    out = []
    for cin, cout, hw, n_pre, n_res in WINO_MIX:
        x = torch.randn(batch, cin, hw, hw, device=dev, generator=g)
        w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) / (3 * cin ** 0.5)
        b = torch.randn(cout, device=dev, generator=g)
        pre = torch.stack([torch.rand(batch, cin, device=dev, generator=g) + 0.5,
                           torch.randn(batch, cin, device=dev, generator=g) * 0.1], -1).contiguous()
        skip = torch.randn(batch, cout, hw, hw, device=dev, generator=g)
        with torch.cuda.stream(st):
            filter_transform(w)
            t_pre = time_kernel(lambda: conv3x3(x, w, b, pre=pre, stats=True), st, reps)
            t_res = time_kernel(lambda: conv3x3(x, w, b, skip=skip, div=2 ** 0.5, pre=pre, stats=True),
                                st, reps)
        fl = 2.0 * batch * cin * cout * 16 * (hw // 2) ** 2  # executed MFMA FLOPs (Winograd)
        out.append(dict(cin=cin, cout=cout, hw=hw, n_pre=n_pre, n_res=n_res, t_pre=t_pre,
                        t_res=t_res, flop=fl))
        del x, skip
    return out


def conv_roofline(dev, batch):
    """achieved = executed MFMA FLOPs of one forward's PRE-conv mix / its HIP-event time.
    Winograd F(2,3) multiplies 16 transformed values per 2x2 output tile per (cin, cout):
    2 * B * Cin * Cout * 16 * (H/2)(W/2) FLOPs per launch = 4/9 of the direct convolution
    (`direct_equivalent_tflops` restates the time on the direct count)."""
    rows = wino_mix_times(dev, batch)
    t = sum(r["n_pre"] * r["t_pre"] + r["n_res"] * r["t_res"] for r in rows)
    fl = sum((r["n_pre"] + r["n_res"]) * r["flop"] for r in rows)
    n_launch = sum(r["n_pre"] + r["n_res"] for r in rows)
    ach = fl / t / 1e12
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
            "traffic": _pmc("wino_pre_mix") if batch == 64 else None,
            "traffic_unit": "HBM bytes per forward mix (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
            "algorithmic_bytes": sum((r["n_pre"] + r["n_res"]) * 4.0 * batch * (r["cin"] + r["cout"]) * r["hw"] ** 2
                                     + r["n_res"] * 4.0 * batch * r["cout"] * r["hw"] ** 2 for r in rows),
            "kernel": "wino_f23_k16_kernel<true> (GroupNorm+SiLU prologue; 8 waves x 16 couts, "
                      "16-input-channel chunks): the NCSN++ 128x128 forward's PRE-conv mix -- bias + "
                      "GN partial statistics, and the residual tail + statistics; "
                      f"{n_launch} launches, B={batch}",
            "flop_basis": "executed (Winograd, 4/9 of direct)",
            "ms_per_mix": round(t * 1e3, 3), "flop_per_mix": fl,
            "direct_equivalent_tflops": round(fl * 9 / 4 / t / 1e12, 2),
            "per_shape": [dict(shape=f"{r['cin']}->{r['cout']}@{r['hw']}",
                               pre_ms=round(r["t_pre"] * 1e3, 4), res_ms=round(r["t_res"] * 1e3, 4),
                               pre_tflops=round(r["flop"] / r["t_pre"] / 1e12, 1))
                          for r in rows]}


# SURVEY.md 8(d) upfirdn2d shapes (B = 64), k = outer([1,3,3,1])/64 (x4 for up)
UPFIRDN_SHAPES = [("down2 [64,128,128,128] pad(1,1)", (128, 128), dict(down=2, pad=(1, 1)), 1.0),
                  ("up2 [64,256,64,64] pad(2,1)", (256, 64), dict(up=2, pad=(2, 1)), 4.0),
                  ("down2 [64,256,64,64] pad(1,1)", (256, 64), dict(down=2, pad=(1, 1)), 1.0),
                  ("fir [64,128,64,64] pad(2,2)", (128, 64), dict(pad=(2, 2)), 1.0)]


def _upfirdn_out(hw, kw):
    up, down = kw.get("up", 1), kw.get("down", 1)
    p0, p1 = kw["pad"]
    return (hw * up + p0 + p1 - 4) // down + 1


def upfirdn_rooflines(dev, batch):
    """HBM roofline of upfirdn2d on the four 8(d) shapes: bytes = 4 (in + out) per launch;
    duration = HIP events around graph replays of 20 launches (time_kernel_graph)."""
    from op import upfirdn2d
    k = torch.tensor(np.outer([1, 3, 3, 1], [1, 3, 3, 1]) / 64.0, dtype=torch.float32, device=dev)
    st = torch.cuda.Stream(dev)
    res = []
    for name, (c, hw), kw, gain in UPFIRDN_SHAPES:
        x = torch.randn(batch, c, hw, hw, device=dev)
        kg = (k * gain).contiguous()  # the scaled taps outside the timed launches
        t = time_kernel_graph(lambda: upfirdn2d(x, kg, **kw), st)
        ho = _upfirdn_out(hw, kw)
        nbytes = 4.0 * (x.numel() + batch * c * ho * ho)
        ach = nbytes / t / 1e9
        res.append({"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": _pmc("upfirdn2d " + name) if batch == 64 else None,
                    "kernel": "upfirdn2d " + name, "ms_per_launch": round(t * 1e3, 4),
                    "bytes_per_launch": nbytes})
        del x
    return res


def cpu_upfirdn_baseline():
    """The reference CPU path's own op sequence (oracle.upfirdn2d_ref.upfirdn2d_native_seq:
    zero insertion by padding, crop, a single-channel conv2d at full resolution, then the
    [::down] slice -- reference op/upfirdn2d.py:159-200) on bounded samples of the four 8(d)
    shapes (batch 4 instead of 64), best of 5, algorithmic GB/s.  (Round 4 timed a strided-conv
    restatement instead: oneDNN ran the 1-channel down2 conv of [1024, 1, 66, 66] planes on a
    direct kernel and the other shapes on its generic path, one shape at 40 GB/s and the rest at
    0.4-1.5.)"""
    from oracle.upfirdn2d_ref import upfirdn2d_native_seq as upfirdn2d_torch
    k = torch.tensor(np.outer([1, 3, 3, 1], [1, 3, 3, 1]) / 64.0, dtype=torch.float32)
    res = {}
    for name, (c, hw), kw, gain in UPFIRDN_SHAPES:
        x = torch.randn(4, c, hw, hw)
        best = 1e9
        for _ in range(5):
            t0 = time.perf_counter()
            y = upfirdn2d_torch(x, k * gain, kw.get("up", 1), kw.get("down", 1), kw["pad"])
            best = min(best, time.perf_counter() - t0)
        res[name] = round(4.0 * (x.numel() + y.numel()) / best / 1e9, 3)
    return {"value": res, "unit": "GB/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": "oracle.upfirdn2d_ref.upfirdn2d_native_seq (the reference's CPU op sequence) "
                      "on the 8(d) shapes at batch 4, best of 5"}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _cpu_threads():
    cores = len(os.sched_getaffinity(0))
    return min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))


def cpu_baseline(n_samples):
    """The oracle (torch-CPU restatement of the reference path, same aten op sequence) on the
    host cores: one warm-up PC step on n_samples (the timed shapes: oneDNN builds its
    primitives per shape), then 1 timed PC step (EM + Langevin = 2 evals per sample) on the
    same n_samples.  Deviation from SURVEY 8(d)'s plan (B = 64 x 3 steps = 384 evals, ~5 min
    at ~1.3 evals/s): a bounded 2 x n_samples-eval sample keeps the default bench within
    minutes; evals/s does not depend on the number of steps."""
    from configs.vp import nc_ncsnpp_128
    from oracle import nets_ref, score_sde_ref
    import models  # noqa: F401
    from models import utils as mutils
    cores = _cpu_threads()
    torch.set_num_threads(cores)
    c = nc_ncsnpp_128.get_config()
    c.device = "cpu"
    torch.manual_seed(0)
    params = nets_ref.init_params(mutils.create_model(c, wrap=False).state_dict())
    sde = score_sde_ref.SDESpec("vp", N=1000)
    mf = lambda x, t: nets_ref.forward(params, c, x, t)
    score_sde_ref.pc_sample(mf, sde, torch.randn(n_samples, 1, 128, 128), "euler_maruyama",
                            "langevin", 0.075, 1, True, n_iters=1)
    t0 = time.perf_counter()
    score_sde_ref.pc_sample(mf, sde, torch.randn(n_samples, 1, 128, 128), "euler_maruyama",
                            "langevin", 0.075, 1, True, n_iters=1)
    dt = time.perf_counter() - t0
    return {"value": round(2 * n_samples / dt, 4), "unit": "score-net evals/s", "cores": cores,
            "kind": "port", "cpu": _cpu_model(),
            "sample": f"oracle/nets_ref + score_sde_ref: 1 PC step (EM+Langevin) on {n_samples} "
                      f"samples of 128x128x1 = {2 * n_samples} evals in {dt:.1f}s after a warm-up "
                      "step at the same batch (plan: B=64 x 3 steps; bounded sample, same "
                      "per-eval work)"}


def cpu_train_baselines():
    """The oracle's DSM train step on the host cores: nets_ref forward (same aten op sequence
    as the reference) + autograd backward + torch Adam + EMA, continuous VP-SDE loss
    (score_sde_ref.dsm_loss).  Bounded samples: NCSN++ 128x128x1 at B=1 (1 warm-up + 1 timed
    step), CIFAR-10 NCSN++ 32x32x3 at B=4 (1 + 2).  Unit: samples/s (and steps/s at that
    batch)."""
    from configs.vp import cifar10_ncsnpp_continuous, nc_ncsnpp_128
    from oracle import nets_ref, score_sde_ref
    import models  # noqa: F401
    from models import utils as mutils
    cores = _cpu_threads()
    torch.set_num_threads(cores)
    out = {}
    for key, mod, B, C, n, steps in (("ncsnpp128", nc_ncsnpp_128, 1, 1, 128, 1),
                                     ("cifar", cifar10_ncsnpp_continuous, 4, 3, 32, 2)):
        c = mod.get_config()
        c.device = "cpu"
        c.model.dropout = 0.0
        torch.manual_seed(0)
        params = nets_ref.init_params(mutils.create_model(c, wrap=False).state_dict())
        leaves = [v for v in params.values() if isinstance(v, torch.Tensor) and v.is_floating_point()]
        for v in leaves:
            v.requires_grad_(True)
        opt = torch.optim.Adam(leaves, lr=2e-4)
        ema = [v.detach().clone() for v in leaves]
        sde = score_sde_ref.SDESpec("vp", N=1000)
        mf = lambda x, t: nets_ref.forward(params, c, x, t)
        x = torch.rand(B, C, n, n)

        def step():
            opt.zero_grad()
            t = torch.rand(B) * (1 - 1e-5) + 1e-5
            loss = score_sde_ref.dsm_loss(mf, sde, x, t, torch.randn_like(x))
            loss.backward()
            torch.nn.utils.clip_grad_norm_(leaves, 1.0)
            opt.step()
            with torch.no_grad():
                for e, v in zip(ema, leaves):
                    e.mul_(0.999).add_(v.detach(), alpha=0.001)
        step()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        dt = (time.perf_counter() - t0) / steps
        out[key] = {"value": round(B / dt, 4), "unit": "train samples/s",
                    "steps_per_s": round(1 / dt, 4), "batch": B, "cores": cores, "kind": "port",
                    "sample": f"oracle nets_ref DSM step ({key}) at B={B}: 1 warm-up + {steps} "
                              f"timed, {dt:.1f}s/step"}
    return out


def cpu_pinn_baseline(B=16, steps=3):
    """The oracle PINN (oracle/pinn_ref.py: FlowNet + PressureNet on aten CPU ops with the
    restated correlation and grid_sample double backward, pinned against the reference
    fixtures by tests/test_pinn_ref.py) trained one configs[3] step at a time on the host
    cores: data losses + pinn_loss_weight x equation_mse, backward, two Adams, EMA.  Bounded
    sample: B = 16 (instead of 64), 1 warm-up + `steps` timed."""
    from configs.pinn import pinn_pde
    from oracle import pinn_ref
    from pinn_kalman.pinn import PINN
    cores = _cpu_threads()
    torch.set_num_threads(cores)
    c = pinn_pde.get_config()
    c.device = torch.device("cpu")
    torch.manual_seed(0)
    P = pinn_ref.init_params(PINN(c).state_dict())
    fl = [v for k, v in P.items() if k.startswith("flownet.")]
    pr = [v for k, v in P.items() if k.startswith("pressurenet.")]
    opt_f, opt_p = torch.optim.Adam(fl, lr=1e-3), torch.optim.Adam(pr, lr=5e-3)
    ema = [v.detach().clone() for v in fl + pr]
    g = torch.Generator().manual_seed(0)
    n = c.data.image_size
    lin = torch.linspace(0.05, 1.0, n)
    f1, f2 = torch.rand(B, 1, n, n, generator=g), torch.rand(B, 1, n, n, generator=g)
    x = (lin.view(1, 1, 1, n) + 0.01 * torch.rand(B, 1, n, n, generator=g)).requires_grad_()
    y = (lin.view(1, 1, n, 1) + 0.01 * torch.rand(B, 1, n, n, generator=g)).requires_grad_()
    t = torch.randint(300, 900, (B,), generator=g).float().requires_grad_()
    target = torch.randn(B, 3, n, n, generator=g) * 0.5
    mask = (torch.rand(B, 1, n, n, generator=g) > 0.1).float()

    def step():
        opt_f.zero_grad()
        opt_p.zero_grad()
        noise = (torch.randn(B, 1, n, n), torch.randn(B, 1, n, n))
        loss, _, _ = pinn_ref.pinn_loss(P, c, (f1, f2, x, y, t, target), mask, noise)
        loss.backward()
        opt_f.step()
        opt_p.step()
        with torch.no_grad():
            for e, v in zip(ema, fl + pr):
                e.mul_(0.9).add_(v.detach(), alpha=0.1)
    step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = (time.perf_counter() - t0) / steps
    return {"value": round(B / dt, 4), "unit": "train samples/s", "steps_per_s": round(1 / dt, 4),
            "batch": B, "cores": cores, "kind": "port",
            "sample": f"oracle/pinn_ref PINN step (configs[3] pinn_pde 64x64) at B={B}: 1 warm-up "
                      f"+ {steps} timed, {dt:.2f}s/step"}


def cpu_dps_baseline(nfe=1):
    """One DPS function evaluation (reference inverse/conditional_sampling.py:100-169: score
    forward, x0_hat, inpainting residual norm, input gradient through the net, drift) on the
    oracle ddpm net (oracle/nets_ref.py, the reference's aten op sequence) at 256x256 on the
    host cores.  Bounded sample: B = 1 (instead of 16), 1 warm-up + `nfe` timed evaluations;
    unit sample-NFE/s."""
    from configs.vp import nc_ddpmpp
    from oracle import nets_ref, score_sde_ref
    import models  # noqa: F401
    from models import utils as mutils
    cores = _cpu_threads()
    torch.set_num_threads(cores)
    c = nc_ddpmpp.get_config()
    c.data.image_size = 256
    c.device = "cpu"
    torch.manual_seed(0)
    params = nets_ref.init_params(mutils.create_model(c, wrap=False).state_dict())
    sde = score_sde_ref.SDESpec("vp", N=c.model.num_scales, beta_min=c.model.beta_min,
                                beta_max=c.model.beta_max)
    score = score_sde_ref.make_score(lambda v, tt: nets_ref.forward(params, c, v, tt), sde, True)
    g = torch.Generator().manual_seed(0)
    n = 256
    mask = (torch.rand(1, 1, n, n, generator=g) > 0.5).float()
    obs = mask * torch.rand(1, 1, n, n, generator=g)
    x = torch.randn(1, 1, n, n, generator=g)
    t = torch.full((1,), 0.5)

    def one():
        xt = x.detach().requires_grad_()
        sc = score(xt, t)
        mean, std = sde.marginal_mean_coef(t), sde.marginal_std(t)
        x0 = xt / mean[:, None, None, None] + std[:, None, None, None] ** 2 * sc
        diff = obs - mask * x0
        norm = torch.linalg.norm(diff)
        gr = torch.autograd.grad(-norm ** 2 / 0.1, xt)[0] / norm.detach()
        dc, dif = sde.coefficient(t)
        return dc[:, None, None, None] * x - dif[:, None, None, None] ** 2 * (sc.detach() + gr) * 0.5
    one()
    t0 = time.perf_counter()
    for _ in range(nfe):
        one()
    dt = (time.perf_counter() - t0) / nfe
    return {"value": round(1 / dt, 4), "unit": "sample-NFE/s", "cores": cores, "kind": "port",
            "sample": f"oracle nets_ref ddpm 256x256 DPS evaluation (forward + input gradient) "
                      f"at B=1: 1 warm-up + {nfe} timed, {dt:.2f}s each"}


def cpu_ns_baseline(steps=100):
    """The C restatement of the reference ns_step (oracle/ns_step_ref.c) on the host cores:
    one 192x192 replica per thread (ctypes releases the GIL inside the C calls, so the
    replicas -- independent, as the simulator's batch -- run in parallel), 1 warm-up + `steps`
    timed full steps (velocity, pressure, density)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import ns_step_ref
    cores = _cpu_threads()
    f, v, p = _ns_fields(np.random.default_rng(0), cores, 192)

    def run(b, k):
        cur = (f[b:b + 1].copy(), v[b:b + 1].copy(), p[b:b + 1].copy())
        for _ in range(k):
            cur = ns_step_ref.full_step(*cur, 0.0025, 0.005)
        return cur

    with ThreadPoolExecutor(cores) as ex:
        list(ex.map(lambda b: run(b, 1), range(cores)))
        t0 = time.perf_counter()
        list(ex.map(lambda b: run(b, steps), range(cores)))
        dt = time.perf_counter() - t0
    return {"value": round(steps * cores * 192 * 192 / dt / 1e9, 4), "unit": "Gsite/s",
            "cores": cores, "kind": "port",
            "sample": f"oracle/ns_step_ref.c (gcc -O2): {cores} replicas of 192^2, one per thread, "
                      f"{steps} full steps each after 1 warm-up, {dt:.2f}s"}


def _ns_fields(rng, B, n):
    """SURVEY.md 8(d) cfg #4 fields: f ~ U(0.1, 1), p ~ N(0, 0.01), u, v ~ U(0.05, 0.5) with a
    random sign (|value| >= 0.05: no exact zero, which is NaN in the reference CIP)."""
    f = rng.uniform(0.1, 1.0, (B, 1, n, n)).astype(np.float32)
    p = rng.normal(0, 0.01, (B, 1, n, n)).astype(np.float32)
    v = (rng.uniform(0.05, 0.5, (B, 2, n, n)) * rng.choice([-1.0, 1.0], (B, 2, n, n))).astype(np.float32)
    return f, v, p


def bench_ns_step(args, ctx, dev):
    """configs[3]'s simulator workload (SURVEY.md 8(d) cfg #4): ns_step full step (velocity,
    pressure, density; two fused launches) on B = 256 replicas of 192x192 per GPU,
    dt = 0.0025, dx = 0.005.  Unit: site-updates/s.  HBM roofline at the algorithmic
    32 B/site (read f, u, v, p; write f, u, v, p); the kernels are VALU-bound by the
    reference-exact arithmetic (fp64 CIP terms, correctly rounded divisions)."""
    from op import ns_step
    B, n = 256, 192
    f, v, p = (torch.tensor(a, device=dev) for a in _ns_fields(np.random.default_rng(ctx.rank), B, n))
    bufs = [(torch.empty_like(f), torch.empty_like(v), torch.empty_like(p)) for _ in range(2)]
    st = torch.cuda.Stream(dev)
    steps = args.ns_steps

    def run(k):
        cur = (f, v, p)
        for i in range(k):
            cur = ns_step.full_step(*cur, 0.0025, 0.005, out=bufs[i % 2])
        return cur

    with torch.cuda.stream(st):
        run(3)
    st.synchronize()
    ctx.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    with torch.cuda.stream(st):
        e0.record(st)
        run(steps)
        e1.record(st)
    st.synchronize()
    ctx.barrier()
    dt = ctx.all_reduce_max(time.perf_counter() - t0, dev)
    t_step = e0.elapsed_time(e1) / 1e3 / steps
    sites = B * n * n
    gbs = 32.0 * sites / t_step / 1e9
    return {"ns_gsites_per_s": round(sites * steps * ctx.world_size / dt / 1e9, 3),
            "ns_ms_per_step": round(t_step * 1e3, 4),
            "ns_config": "configs[3] simulator: ns_step full step, 256 x 192x192 per GPU",
            "roofline_ns_step": {"bound": "valu (reference-exact fp64/division arithmetic)",
                                 "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(gbs / HBM_PEAK_GBS, 4),
                                 "traffic": _pmc("ns_step full step B256 192^2"),
                                 "kernel": "ns_step fused velocity + pressure/density launches",
                                 "bytes_per_step": 32.0 * sites},
            "roofline_ns_step_valu": _ns_valu_roofline(t_step)}


def _ns_valu_roofline(t_step):
    cyc, src = _ns_valu_cycles()
    if cyc is None:
        return None
    peak = 1024 * 2.4e9  # SIMD-cycles/s: 256 CUs x 4 SIMDs at the 2.4 GHz max clock
    ach = cyc / t_step
    return {"bound": "valu", "achieved": round(ach / 1e12, 4), "peak": round(peak / 1e12, 4),
            "unit": "T SIMD-issue-cycles/s", "frac": round(ach / peak, 4), "traffic": None,
            "kernel": "ns_step full step (velocity + pressure/density launches)",
            "profile_derived": src,
            "basis": f"VALU-active SIMD-cycles per step {cyc:.4g} (SQ_ACTIVE_INST_VALU x 4 from the "
                     f"PMC pass {src} of these kernel sources) / live step time, vs 1024 SIMDs x "
                     "2.4 GHz"}


def bench_ncddpmpp(args, ctx, dev):
    """The literal configs[2] variant: configs/vp/nc_ddpmpp.py at 128x128x1
    (model `ddpm`, discrete VP, ancestral_sampling predictor, no corrector), B = 64 per GPU,
    graph-replayed PC steps; 1 score evaluation per sample per step."""
    import models  # noqa: F401
    import sampling
    import sde_lib
    from configs.vp import nc_ddpmpp
    from models import utils as mutils
    c = nc_ddpmpp.get_config()
    c.data.image_size = 128
    c.device = dev
    torch.manual_seed(0)
    model = mutils.create_model(c, wrap=False).eval()
    with torch.no_grad():
        for prm in model.parameters():
            prm.add_(torch.randn_like(prm) * 0.01)
    B = shard(args, ctx.world_size, args.global_batch)
    sde = sde_lib.VPSDE(c.model.beta_min, c.model.beta_max, c.model.num_scales)
    eng = sampling.PCEngine(sde, (B, 1, 128, 128), sampling.AncestralSamplingPredictor,
                            sampling.NoneCorrector, c.sampling.snr, 1, continuous=False,
                            device=dev, seed=4321, dist_ctx=ctx if ctx.world_size > 1 else None)
    eng.reset(model)
    eng.advance(2)
    torch.cuda.synchronize(dev)
    ctx.barrier()
    t0 = time.perf_counter()
    eng.advance(args.ncddpmpp_steps)
    torch.cuda.synchronize(dev)
    ctx.barrier()
    dt = ctx.all_reduce_max(time.perf_counter() - t0, dev)
    return {"ncddpmpp_evals_per_s": round(B * ctx.world_size * args.ncddpmpp_steps / dt, 2),
            "ncddpmpp_ms_per_step": round(dt / args.ncddpmpp_steps * 1e3, 2),
            "ncddpmpp_tflops": round(B * ctx.world_size * args.ncddpmpp_steps * 300.53e9 / dt / 1e12, 2),
            "ncddpmpp_config": "configs[2] literal: nc_ddpmpp (ddpm, 300.53 GFLOP/eval) 128x128x1, "
                               f"ancestral + none, discrete, global batch {B * ctx.world_size}, "
                               f"{B}/GPU"}


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
    B = shard(args, ctx.world_size, c.training.batch_size, explicit=False)
    batch = torch.rand(B, 3, 32, 32, device=dev, generator=torch.Generator(device=dev).manual_seed(ctx.rank))
    for _ in range(2):
        step_fn(state, batch)
    tally, _ = counted(lambda: step_fn(state, batch), dev)
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
            "cifar_config": f"configs[1]: cifar10_ncsnpp_continuous 32x32x3, global batch "
                            f"{B * ctx.world_size}, {B}/GPU",
            "roofline_cifar_train": step_roofline(
                tally, args.cifar_steps / dt, "configs[1] DSM train step, NCSN++ CIFAR-10 32x32x3 "
                f"B={B}/GPU", survey_direct=8.36e12 * B / 128,
                traffic_key="step cifar" if B == 128 else None)}


def _pinn_run(args, ctx, dev):
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
    eager_fn = losses.get_pinn_step_fn(c, train=True, optimize_fn=losses.optimization_manager(c),
                                       ctx=ctx)
    step_fn = eager_fn if args.pinn_eager else losses.get_pinn_step_fn(
        c, train=True, optimize_fn=losses.optimization_manager(c), ctx=ctx, graph=True)
    B = shard(args, ctx.world_size, c.training.batch_size)
    c.training.batch_size = B  # the per-rank batch: the observation masks are [B, 1, H, W]
    operator = get_operator(c)
    batch = pinn_batch(c, B, dev, seed=ctx.rank)
    if args.pinn_eager:  # the eager step's conv choices (their timing runs) before the count
        eager_fn(state, operator, batch)
    for _ in range(args.pinn_warmup):  # the first graph-mode call captures the step
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
    losses_ = tuple(float(v) for v in (loss, pinn_loss, data_loss))
    # FLOPs of one step: counted on an eager step (a graph replay launches nothing from
    # Python), after the timed region -- an eager step before the capture left later replays
    # reading garbage on this stack (tools/diag_pinn_bench.py), and the graph's warm-up made
    # the conv choices already
    tally, _ = counted(lambda: eager_fn(state, operator, batch), dev)
    return dt, losses_, tally, B


def bench_pinn(args, ctx, dev):
    """configs[3]: one PINN train step (get_pinn_step_fn: FlowNet + PressureNet forward,
    equation_mse with create_graph first derivatives and second derivatives -- correlation,
    grid_sample grad2 and the InstanceNorm+ELU double backward on HIP --, backward, two
    Adams, EMA) at pinn_pde, global batch 64 sharded over the ranks, 64x64; gradients averaged
    over ranks with RCCL.
    The step's forward + backward replayed from one hipGraph (losses.get_pinn_step_fn(
    graph=True)); --pinn-eager times the eager step."""
    dt, losses_, tally, B = _pinn_run(args, ctx, dev)
    roof = None
    if tally is not None:
        roof = step_roofline(tally, args.pinn_steps / dt, "configs[3] PINN train step (FlowNet + "
                             "PressureNet fwd, equation_mse 1st/2nd derivatives, backward, 2x Adam, "
                             f"EMA), B={B}/GPU 64x64; latency-bound: ~10k launches per step",
                             traffic_key="step pinn")
        roof["bound_note"] = ("mfma is the nominal bound; the step is launch/latency-bound (small "
                              "images, ~10k kernels), so frac is low by construction")
    return {"roofline_pinn": roof, "pinn_train_steps_per_s": round(args.pinn_steps / dt, 3),
            "pinn_ms_per_step": round(dt / args.pinn_steps * 1e3, 2),
            "pinn_mode": "eager" if args.pinn_eager else "hip_graph",
            "pinn_global_batch": B * ctx.world_size,
            "pinn_losses": [round(v, 6) for v in losses_],
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
    c.training.batch_size = shard(args, ctx.world_size, 16, explicit=False)
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
    from models.utils import input_grad_only
    f = sampler.make_ode_func(model)

    def one_nfe():
        with input_grad_only(model):
            return f(0.5, z.reshape(-1).to(torch.float64))
    tally, _ = counted(one_nfe, dev)
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
            "dps_config": f"configs[4]: nc_ddpmpp_inpaint_dps @256x256 (ddpm net), global batch "
                          f"{B * ctx.world_size}, {B}/GPU, RK45",
            "roofline_dps": step_roofline(tally, nfe / dt, "configs[4] DPS function evaluation "
                                          f"(ddpm 256x256 forward + input gradient through the net, "
                                          f"B={B}/GPU)", unit_of_work="nfe",
                                          survey_direct=2 * 1198.88e9 * B,
                                          traffic_key="step dps" if B == 16 else None)}


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


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`python bench.py --gpus N` (N > 1) outside torchrun: start N ranks, one per GPU, as
    `torch.distributed.run` in a child process (this process never touches the GPU), relay
    rank 0's JSON line to stdout and exit with the launcher's status.  The reference reaches
    every visible GPU from one command too (nn.DataParallel, models/utils.py:93)."""
    backend = os.environ.get("BPK_DIST_BACKEND", "nccl")
    if backend == "nccl" and not args.plumbing:
        have = torch.cuda.device_count()  # no HIP context is created by this call
        if have < args.gpus:
            print(f"[bench] --gpus {args.gpus} but only {have} GPU(s) visible "
                  "(BPK_DIST_BACKEND=gloo rehearses several ranks on one device)",
                  file=sys.stderr, flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"launching {args.gpus} ranks: {' '.join(cmd[1:6])} ...")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    line = None
    for out in proc.stdout:
        if out.startswith("{") and '"metric"' in out:
            line = out.strip()
        else:
            sys.stderr.write(out)
            sys.stderr.flush()
    rc = proc.wait()
    if rc == 0 and line is None:
        print("[bench] ranks exited 0 but rank 0 printed no result line", file=sys.stderr)
        rc = 1
    if line is not None:
        print(line, flush=True)
    return rc


def _plumbing(args, ctx):
    """--plumbing: the multi-rank launch path without GPU work (CPU tests, gloo)."""
    t = torch.tensor([float(ctx.rank + 1)], dtype=torch.float64)
    if ctx.world_size > 1:
        torch.distributed.all_reduce(t)
    if ctx.rank == 0:
        print(json.dumps({"metric": "plumbing", "value": float(t.item()), "n_gpus": ctx.world_size,
                          "per_gpu_batch": shard(args, ctx.world_size, args.global_batch),
                          "scaling": scaling_mode(args),
                          "backend": torch.distributed.get_backend() if ctx.world_size > 1 else None}),
              flush=True)
    if ctx.world_size > 1:
        torch.distributed.destroy_process_group()


def main():
    args = parse()
    _heartbeat()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if world_env is not None and int(world_env) != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world_env}: refusing a mismatched "
              "launch", file=sys.stderr, flush=True)
        sys.exit(2)
    import dist
    if args.plumbing:
        return _plumbing(args, dist.init_from_env(
            backend=os.environ.get("BPK_DIST_BACKEND", "gloo")))
    import sampling
    import sde_lib
    ctx = dist.init_from_env()
    torch.backends.cudnn.benchmark = bool(args.miopen_find)
    # one rank per GPU; more ranks than devices only in a gloo rehearsal on one box
    dev = torch.device("cuda", ctx.local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    world = ctx.world_size
    B = shard(args, world, args.global_batch)
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

    sums = None
    if args.sample_sums:
        sums = ctx.all_gather_cat(x.double().sum(dim=(1, 2, 3))).cpu().tolist()

    roof = None
    if ctx.rank == 0 and not args.no_roofline:
        log("dominant-kernel roofline (right after the sampler: same clock regime)")
        from op.conv import local_choices
        with local_choices():  # rank 0 only: no collective may start in here
            roof = conv_roofline(dev, B)

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
        tally, _ = counted(lambda: step_fn(state, batch), dev)
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
                 "train_tflops_direct_basis": round(args.train_steps * B * world * NCSNPP_GFLOP_PER_TRAIN_SAMPLE
                                                    / tdt / 1e3, 2),
                 "roofline_train": step_roofline(
                     tally, args.train_steps / tdt, f"configs[2] DSM train step, NCSN++ 128x128x1 B={B}/GPU "
                     "(fwd + bwd-data + wgrad + clip + Adam + EMA)", survey_direct=63.9e12 * B / 64,
                     traffic_key="step train" if B == 64 else None)}

    cifar = None
    if args.cifar_steps > 0 and not args.no_train:
        log("configs[1] train steps (CIFAR-10 32x32, batch 128)")
        _phase_reset(dev)
        cifar = bench_cifar_train(args, ctx, dev)

    pinn = None
    if not args.no_pinn:
        log("PINN train steps")
        _phase_reset(dev)
        pinn = bench_pinn(args, ctx, dev)

    dps = None
    if not args.no_dps:
        log("DPS function evaluations")
        _phase_reset(dev)
        dps = bench_dps(args, ctx, dev)

    ns = None
    if args.ns_steps > 0:
        log("ns_step simulator steps")
        ns = bench_ns_step(args, ctx, dev)

    ncd = None
    if args.ncddpmpp_steps > 0:
        log("nc_ddpmpp 128^2 ancestral sampler")
        ncd = bench_ncddpmpp(args, ctx, dev)

    result = None
    if ctx.rank == 0:
        up_roof = None
        if not args.no_roofline:
            log("upfirdn2d rooflines")
            from op.conv import local_choices
            with local_choices():
                up_roof = upfirdn_rooflines(dev, 64)  # the 8(d) shapes, whatever the sharding
        model_tflops = evals_per_s * NCSNPP_GFLOP_PER_EVAL / 1e3
        result = {
            "metric": "PC-sampler score-net evals/s (NCSN++ 128x128x1, EM + Langevin)",
            "value": round(evals_per_s, 3), "unit": "score-net evals/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": scaling_mode(args), "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (prior noise, random-init weights)",
            "config": {"workload": "configs[2]: NCSN++ 128x128x1 PC sampler, VP-SDE N=1000, "
                                   f"euler_maruyama + langevin (snr 0.075), global batch {B * world} "
                                   f"= {B}/GPU x {world}",
                       "model": "ncsnpp (62.69M params)", "global_batch": B * world,
                       "per_gpu_batch": B,
                       "per_rank_of_n_gpus": args.per_rank_of,
                       "seq_len": None, "parallelism": f"dp{world} (batch-sharded, RCCL)",
                       "hip_graph": eng.graph is not None,
                       "dist_backend": torch.distributed.get_backend() if world > 1 else None,
                       "pc_graph_allreduce": bool(world > 1 and sampling._graph_collective(ctx))},
            "score_net_tflops": round(model_tflops, 2),
            "score_net_tflops_basis": "direct-conv FLOP count (333.25 GFLOP/eval, SURVEY 8d); "
                                      "the Winograd convs execute 4/9 of its 3x3 multiplies, so "
                                      "this rate may exceed the MFMA peak",
            "samples_finite": finite,
            "roofline": roof,
            "roofline_upfirdn2d": up_roof,
        }
        if sums is not None:
            result["sample_sums"] = sums
        for part in (train, cifar, pinn, dps, ns, ncd):
            if part:
                result.update(part)
    if world == 1 and not args.no_cpu_baseline and ctx.rank == 0:
        log("cpu baseline")
        result["cpu_baseline"] = cpu_baseline(args.cpu_samples)
        result["speedup_vs_cpu"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
        log("cpu baselines of the other rows")
        extra = {"upfirdn2d": cpu_upfirdn_baseline(), "ns_step": cpu_ns_baseline()}
        if not args.no_train:
            extra.update(cpu_train_baselines())
        if not args.no_pinn:
            extra["pinn"] = cpu_pinn_baseline()
        if not args.no_dps:
            extra["dps"] = cpu_dps_baseline()
        result["cpu_baselines_other"] = extra
    if ctx.rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
