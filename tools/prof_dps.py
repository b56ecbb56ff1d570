"""configs[4] DPS function evaluations alone (bench.bench_dps: nc_ddpmpp 256x256 ddpm net, B=16,
RK45), for a rocprofv3 --kernel-trace --stats summary of DPS NFEs without the PC-sampler phase
of a full bench run.  argv[1]: accepted RK45 steps timed (default 2).  Prints bench_dps's dict
plus the total number of function evaluations the process ran (warm-up + counted + timed)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
import dist  # noqa: E402
from inverse.conditional_sampling import get_solver  # noqa: E402

steps = sys.argv[1] if len(sys.argv) > 1 else "2"
sys.argv = ["bench.py", "--dps-steps", steps]
args = bench.parse()
ctx = dist.init_from_env()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
res = bench.bench_dps(args, ctx, dev)
res.pop("roofline_dps", None)
res["note"] = ("process total NFE = warm-up solve (1 accepted step) + 1 counted NFE + the timed "
               "solve's dps_nfe_timed")
print(json.dumps(res), flush=True)
