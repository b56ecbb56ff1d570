"""Defaults for the NetCDF ocean-field runs (reference configs/default_nc_configs.py:5-76)."""
import torch

from configs._configdict import ConfigDict


def get_default_configs():
    c = ConfigDict()
    c.training = ConfigDict(dict(batch_size=64, n_iters=50000, snapshot_freq=10000, log_freq=500,
                                 eval_freq=100, snapshot_freq_for_preemption=25000,
                                 snapshot_sampling=True, likelihood_weighting=False,
                                 continuous=True, reduce_mean=False))
    c.sampling = ConfigDict(dict(n_steps_each=1, noise_removal=True, probability_flow=False,
                                 snr=0.075))
    c.eval = ConfigDict(dict(begin_ckpt=50, end_ckpt=96, batch_size=512, enable_sampling=True,
                             num_samples=50000, enable_loss=True, enable_bpd=False,
                             bpd_dataset="test"))
    c.data = ConfigDict(dict(dataset="NC", image_size=64, random_flip=False,
                             uniform_dequantization=False, centered=False, num_channels=1,
                             category="Theta", key="THETA", date_range="2013to2017_1day",
                             depth=0, land_cut=200))
    c.model = ConfigDict(dict(sigma_max=378, sigma_min=0.01, num_scales=2000, beta_min=0.1,
                              beta_max=20., dropout=0., embedding_type="fourier"))
    c.optim = ConfigDict(dict(weight_decay=0, optimizer="Adam", lr=2e-4, beta1=0.9, eps=1e-8,
                              warmup=5000, grad_clip=1.))
    c.seed = 42
    c.device = torch.device("cuda:0") if torch.cuda.is_available() else torch.device("cpu")
    return c
