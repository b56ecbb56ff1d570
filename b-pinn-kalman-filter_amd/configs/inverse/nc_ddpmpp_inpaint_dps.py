"""DPS inpainting on the NetCDF DDPM (BASELINE.json configs[4]) -- reference
configs/inverse/nc_ddpmpp_inpaint_dps.py: nc_ddpmpp + batch 16 + an `inverse` section
(inpaint operator, half the pixels observed, observation variance 0.1, RK45)."""
from configs._configdict import ConfigDict
from configs.vp import nc_ddpmpp


def get_config():
    c = nc_ddpmpp.get_config()
    c.training.batch_size = 16
    c.inverse = ConfigDict(dict(operator="inpaint", invert=False, ratio=0.5, sampler="dps",
                                variance=0.1, solver="RK45"))
    return c
