"""The fork's "DDPM++" config: model 'ddpm' (reference configs/vp/cifar10_ddpmpp_continuous.py:42).
BASELINE.json configs[0] (CPU plumbing)."""
from configs.default_cifar10_configs import get_default_configs


def get_config():
    c = get_default_configs()
    c.training.update(sde="vpsde", continuous=True, reduce_mean=True)
    c.sampling.update(method="pc", predictor="euler_maruyama", corrector="none")
    c.data.centered = True
    c.model.update(name="ddpm", scale_by_sigma=False, ema_rate=0.9999, normalization="GroupNorm",
                   nonlinearity="swish", nf=128, ch_mult=(1, 2, 2, 2), num_res_blocks=4,
                   attn_resolutions=(16,), resamp_with_conv=True, conditional=True, fir=False,
                   fir_kernel=[1, 3, 3, 1], skip_rescale=True, resblock_type="biggan",
                   progressive="none", progressive_input="none", progressive_combine="sum",
                   attention_type="ddpm", init_scale=0., embedding_type="positional",
                   fourier_scale=16, conv_size=3)
    return c
