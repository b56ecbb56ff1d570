"""PINN on the PDE dataset (reference configs/pinn/pinn_pde.py) -- BASELINE configs[3]."""
from configs._configdict import ConfigDict
from configs.pinn.pinn_default_configs import get_default_configs


def get_config():
    c = get_default_configs()
    c.data.dataset = "PDE"
    c.data.dt = 1.7
    c.data.time_trim = 300
    c.inverse = ConfigDict(dict(operator="inpaint_rnd", invert=False, ratio=0.9, variance=0.01))
    c.kf = ConfigDict(dict(patch_size=8))
    return c
