"""PINN graph replay vs eager with NaN-poisoned eager re-allocations between steps, for the
current losses.py and (if tools/_old_losses.py exists) the round-2 version."""
import importlib.util
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import numpy as np
import torch
import test_gpu_pinn as T

dev = torch.device("cuda:0")
mods = [("current", None)]
old = os.path.join(REPO, "tools", "_old_losses.py")
if os.path.exists(old):
    spec = importlib.util.spec_from_file_location("old_losses", old)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    mods.append(("r02", m))
B = int(os.environ.get("B", 2))
for name, mod in mods:
    for poison in (False, True):
        l1, l2, g1, g2 = T.pinn_graph_vs_eager(dev, mod, steps=12, poison=poison, B=B)
        rel = np.abs(np.array(l2) - np.array(l1)) / np.abs(np.array(l1))
        print(name, "poison" if poison else "plain", "max rel loss diff", float(np.nanmax(rel)) if np.isfinite(rel).any() else "nan",
              "grad rel", float((g1 - g2).norm() / g1.norm()), flush=True)
        print("  eager", [round(v, 6) for v in l1], flush=True)
        print("  graph", [round(v, 6) for v in l2], flush=True)
