"""Which convs MIOpen would win: the DSM train step (NCSN++ 128^2, B=64), the CIFAR-10 train
step (B=128) and the PINN eager step (B=64) run once under op.conv.library_candidates(), with
every igemm-vs-MIOpen timing recorded.  Prints one line per decided key: the two times and
the winner, sorted by the time MIOpen saves (x calls per step)."""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

from op import conv  # noqa: E402

rec = {}
calls = collections.Counter()
_orig_decide, _orig_pick = conv._decide, conv._pick


def decide(key, timers):
    if key in conv._CHOICE:
        return conv._CHOICE[key]
    ts = []
    orig_time = conv._time_us

    def timed(f):
        t = orig_time(f)
        ts.append(t)
        return t
    conv._time_us = timed
    try:
        c = _orig_decide(key, timers)
    finally:
        conv._time_us = orig_time
    if ts:
        rec[key] = ts
    return c


def pick(key, run_ig, run_mi):
    calls[key] += 1
    return _orig_pick(key, run_ig, run_mi)


conv._decide = decide
conv._pick = pick
dev = torch.device("cuda:0")
phase = sys.argv[1] if len(sys.argv) > 1 else "train"
with conv.library_candidates():
    if phase == "train":
        import bench
        import losses
        import sde_lib
        from models.ema import ExponentialMovingAverage
        c, model = bench.build_model(dev)
        c.model.dropout = 0.0
        model.train()
        sde = sde_lib.VPSDE(c.model.beta_min, c.model.beta_max, c.model.num_scales)
        opt = losses.get_optimizer(c, model.parameters())
        ema = ExponentialMovingAverage(model.parameters(), decay=c.model.ema_rate)
        state = dict(optimizer=opt, model=model, ema=ema, step=0)
        step_fn = losses.get_step_fn(sde, train=True, optimize_fn=losses.optimization_manager(c),
                                     reduce_mean=True, continuous=True)
        batch = torch.rand(64, 1, 128, 128, device=dev)
        step_fn(state, batch)
        calls.clear()
        step_fn(state, batch)
    else:
        import bench
        from dist import DistContext

        class A:
            pass
        args = A()
        args.batch = None
        args.weak = False
        args.per_rank_of = None
        if phase == "cifar":
            args.cifar_steps = 1
            bench.bench_cifar_train(args, DistContext(), dev)
        else:
            args.pinn_warmup, args.pinn_steps, args.pinn_eager = 0, 1, True
            bench.bench_pinn(args, DistContext(), dev)
torch.cuda.synchronize()
rows = []
for key, ts in rec.items():
    if len(ts) != 2 or key[0] not in ("fwd", "dgrad", "wgrad"):
        continue
    n = max(calls[key], 1)
    rows.append(((ts[0] - ts[1]) * n, key, ts, n))
rows.sort(key=lambda r: -r[0])
tot_ig = sum(r[2][0] * r[3] for r in rows)
tot_best = sum(min(r[2]) * r[3] for r in rows)
print(f"{phase}: {len(rows)} igemm-vs-MIOpen keys; per step igemm {tot_ig / 1e3:.2f} ms, "
      f"best-of {tot_best / 1e3:.2f} ms", flush=True)
for save, key, ts, n in rows:
    print(f"  save {save / 1e3:7.3f} ms  x{n:<3d} igemm {ts[0]:8.1f} us  miopen {ts[1]:8.1f} us  {key}")
