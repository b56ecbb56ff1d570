"""DSM train steps (NCSN++ 128x128x1, B=64 -- or B=argv[1], e.g. 8 for the 8-GPU point's
per-rank work -- the bench's train phase) for rocprofv3: 2 warm-up + 3 profiled steps."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
import bench
import losses
import sde_lib
from models.ema import ExponentialMovingAverage
dev = torch.device("cuda:0")
c, model = bench.build_model(dev)
c.model.dropout = 0.0
model.train()
sde = sde_lib.VPSDE(c.model.beta_min, c.model.beta_max, c.model.num_scales)
opt = losses.get_optimizer(c, model.parameters())
ema = ExponentialMovingAverage(model.parameters(), decay=c.model.ema_rate)
state = dict(optimizer=opt, model=model, ema=ema, step=0)
step_fn = losses.get_step_fn(sde, train=True, optimize_fn=losses.optimization_manager(c),
                             reduce_mean=True, continuous=True)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
batch = torch.rand(B, 1, 128, 128, device=dev)
for i in range(5):
    loss = step_fn(state, batch)
    torch.cuda.synchronize()
    print("step", i, float(loss), flush=True)
