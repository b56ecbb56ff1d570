"""NCSN++ / continuous VP-SDE on CIFAR-10 (reference configs/vp/cifar10_ncsnpp_continuous.py).
BASELINE.json configs[1]."""
from configs.default_cifar10_configs import get_default_configs

NCSNPP_MODEL = dict(name="ncsnpp", scale_by_sigma=False, ema_rate=0.9999,
                    normalization="GroupNorm", nonlinearity="swish", nf=128,
                    ch_mult=(1, 2, 2, 2), num_res_blocks=4, attn_resolutions=(16,),
                    resamp_with_conv=True, conditional=True, fir=True, fir_kernel=[1, 3, 3, 1],
                    skip_rescale=True, resblock_type="biggan", progressive="none",
                    progressive_input="residual", progressive_combine="sum",
                    attention_type="ddpm", embedding_type="positional", init_scale=0.,
                    fourier_scale=16, conv_size=3)


def get_config():
    c = get_default_configs()
    c.training.update(sde="vpsde", continuous=True, reduce_mean=True)
    c.sampling.update(method="pc", predictor="euler_maruyama", corrector="none")
    c.data.centered = True
    c.model.update(NCSNPP_MODEL)
    return c
