"""NetCDF DDPM (model 'ddpm', discrete VP, ancestral sampling) -- reference configs/vp/nc_ddpmpp.py."""
from configs.default_nc_configs import get_default_configs


def get_config():
    c = get_default_configs()
    c.training.update(sde="vpsde", continuous=False, reduce_mean=True)
    c.sampling.update(method="pc", predictor="ancestral_sampling", corrector="none")
    c.data.update(category="Theta", key="THETA", date_range="2013to2017_1day")
    c.model.update(name="ddpm", scale_by_sigma=False, ema_rate=0.9999, normalization="GroupNorm",
                   nonlinearity="swish", nf=128, ch_mult=(1, 2, 2, 2), num_res_blocks=4,
                   attn_resolutions=(16,), resamp_with_conv=True, conditional=True, fir=False,
                   fir_kernel=[1, 3, 3, 1], skip_rescale=True, resblock_type="biggan",
                   progressive="none", progressive_input="none", progressive_combine="sum",
                   attention_type="ddpm", init_scale=0., embedding_type="positional",
                   fourier_scale=16, conv_size=3)
    return c
