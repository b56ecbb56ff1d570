"""rocprofv3 --pmc driver for the whole-step rooflines' HBM traffic: runs one bench phase
(MODE = train | cifar | pinn | dps) through bench.main with one timed step, and brackets the
phase's single counted step (bench.counted: after the warm-up, outside the timed loop) with a
marker dispatch of fused_bias_act_kernel on 256 floats (a kernel no bench phase launches).
tools/pmc_summary.py sums FETCH_SIZE / WRITE_SIZE over the dispatches between the markers.
The PINN phase runs its eager step (--pinn-eager): the counted step is eager in either mode,
and the hipGraph capture of the timed step segfaulted under rocprofv3 --pmc (round 4)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402

MODE = sys.argv[1]
_orig = bench.counted


def _marker(dev):
    from op.fused_act import fused_bias_act_raw
    t = torch.zeros(256, device=dev)
    fused_bias_act_raw(t, None, None, 1, 0, 0.2, 1.0)
    torch.cuda.synchronize(dev)


def counted(fn, dev):
    torch.cuda.synchronize(dev)
    _marker(dev)
    r = _orig(fn, dev)
    _marker(dev)
    return r


bench.counted = counted
common = ["--steps", "1", "--warmup", "1", "--no-roofline", "--no-cpu-baseline", "--ns-steps", "0",
          "--ncddpmpp-steps", "0"]
argv = {"train": ["--train-steps", "1", "--cifar-steps", "0", "--no-pinn", "--no-dps"],
        "cifar": ["--train-steps", "1", "--train-warmup", "0", "--cifar-steps", "1", "--no-pinn",
                  "--no-dps"],
        "pinn": ["--no-train", "--pinn-steps", "1", "--pinn-warmup", "1", "--no-dps", "--pinn-eager"],
        "dps": ["--no-train", "--no-pinn", "--dps-steps", "1"]}[MODE]
sys.argv = ["bench.py"] + common + argv
bench.main()
print("ok", MODE, flush=True)
