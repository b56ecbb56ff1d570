"""diag_pinn_graph5 after the bench's PC-sampler phase in the same process (the bench's order:
NCSN++ 128 model, PCEngine capture + steps), graph vs eager PINN losses per step.  DIAG:
nograph = sampler without its hipGraph; nosampler = skip the sampler phase."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tools"), os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402

T = set(os.environ.get("DIAG", "").split(","))
dev = torch.device("cuda:0")
if "nosampler" not in T:
    import sampling
    import sde_lib
    c, model = bench.build_model(dev)
    model.eval()
    sde = sde_lib.VPSDE(c.model.beta_min, c.model.beta_max, c.model.num_scales)
    eng = sampling.PCEngine(sde, (64, 1, 128, 128), sampling.EulerMaruyamaPredictor,
                            sampling.LangevinCorrector, c.sampling.snr, 1, continuous=True,
                            device=dev, seed=1234, use_graph="nograph" not in T)
    eng.reset(model)
    eng.advance(3)
    torch.cuda.synchronize()
    print("sampler done, graph", eng.graph is not None, flush=True)
import diag_pinn_graph5 as d5  # noqa: E402  (runs eager vs graph and prints)
