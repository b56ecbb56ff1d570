"""Defaults for CIFAR-10 score SDE runs (reference configs/default_cifar10_configs.py:5-72)."""
import torch

from configs._configdict import ConfigDict


def get_default_configs():
    c = ConfigDict()
    c.training = ConfigDict(dict(batch_size=128, n_iters=10001, snapshot_freq=5000, log_freq=50,
                                 eval_freq=100, snapshot_freq_for_preemption=10000,
                                 snapshot_sampling=True, likelihood_weighting=False,
                                 continuous=True, reduce_mean=False))
    c.sampling = ConfigDict(dict(n_steps_each=1, noise_removal=True, probability_flow=False,
                                 snr=0.16))
    c.eval = ConfigDict(dict(begin_ckpt=9, end_ckpt=26, batch_size=1024, enable_sampling=False,
                             num_samples=50000, enable_loss=True, enable_bpd=False,
                             bpd_dataset="test"))
    c.data = ConfigDict(dict(dataset="CIFAR10", image_size=32, random_flip=True, centered=False,
                             uniform_dequantization=False, num_channels=3))
    c.model = ConfigDict(dict(sigma_min=0.01, sigma_max=50, num_scales=1000, beta_min=0.1,
                              beta_max=20., dropout=0.1, embedding_type="fourier"))
    c.optim = ConfigDict(dict(weight_decay=0, optimizer="Adam", lr=2e-4, beta1=0.9, eps=1e-8,
                              warmup=5000, grad_clip=1.))
    c.seed = 42
    c.device = torch.device("cuda:0") if torch.cuda.is_available() else torch.device("cpu")
    return c
