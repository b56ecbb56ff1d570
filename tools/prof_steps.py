"""rocprofv3 --pmc driver for the whole-step rooflines' HBM traffic: runs one bench phase
(MODE = train | cifar | pinn | dps) through bench.main with one timed step, and brackets the
phase's single counted step (bench.counted: after the warm-up, outside the timed loop) with a
marker dispatch of fused_bias_act_kernel<double> on 256 values (an instance no bench phase
launches: FlowNet's LeakyReLU runs the float one).
tools/pmc_summary.py sums FETCH_SIZE / WRITE_SIZE over the dispatches between the markers.
The PINN phase runs its eager step (--pinn-eager): the counted step is eager in either mode.
Under rocprofv3 --pmc the profiler's preloaded library starts the HIP runtime before Python
runs, so DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 must be exported by the shell (op/_hipenv.py cannot set
it in time, and with it unset the graph phases fall back to their eager steps).  Rounds 4-5
ran without it and their PINN / DPS passes died with SIGSEGV inside a kernel launch at a
kernel-argument-pool boundary, sidestepped with HSA_KERNARG_POOL_SIZE=67108864 (DESIGN.md
section 6 for what round 6 found)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
from op import _hipenv  # noqa: E402,F401
import torch  # noqa: E402

import bench  # noqa: E402

MODE = sys.argv[1]
_orig = bench.counted


def _marker(dev):
    from op.fused_act import fused_bias_act_raw
    t = torch.zeros(256, device=dev, dtype=torch.float64)  # the f64 instance: no phase runs it
    fused_bias_act_raw(t, None, None, 1, 0, 0.2, 1.0)
    torch.cuda.synchronize(dev)


def counted(fn, dev):
    torch.cuda.synchronize(dev)
    _marker(dev)
    r = _orig(fn, dev)
    _marker(dev)
    return r


bench.counted = counted
if MODE == "dps":
    # the counted NFE is all the PMC pass needs: the warm-up and the timed RK45 solves become
    # one function evaluation each (every dispatch is serialized under --pmc: the real solves
    # took minutes)
    import inverse.conditional_sampling as _cs

    def _one_eval(config, ode_func, x0, t1, shape, eps, ctx=None):
        _cs.get_solver.last_nfe = 1
        return ode_func(t1, x0).reshape(shape).to(torch.float32)
    _one_eval.last_nfe = 1
    _cs.get_solver = _one_eval
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
