"""Defaults of the PINN runs (reference configs/pinn/pinn_default_configs.py:5-59)."""
import torch

from configs._configdict import ConfigDict


def get_default_configs():
    c = ConfigDict()
    c.training = ConfigDict(dict(batch_size=64, n_iters=35000, n_pinn_iters=25000,
                                 n_bpinn_iters=40000, snapshot_freq=5000,
                                 snapshot_freq_for_preemption=250, log_freq=5, eval_freq=50,
                                 pinn_loss_weight=1e-5))
    c.data = ConfigDict(dict(num_channels=1, dataset="_", image_size=64, random_flip=False,
                             uniform_dequantization=False, centered=False))
    c.model = ConfigDict(dict(ema_rate=0.9, arch="flownet", feature_nums=[16, 32, 64, 96, 128],
                              spatial_embed_omega=100, spatial_embed_s_flow=100,
                              spatial_embed_s_pres=100, bpinn_moped_delta=0.01))
    c.optim = ConfigDict(dict(weight_decay=0, bpinn_weight_decay=0, optimizer="Adam", lr=0.001,
                              bpinn_lr=0.0005, beta1=0.9, eps=1e-8, warmup=100, grad_clip=1.))
    c.seed = 42
    c.device = torch.device("cuda:0") if torch.cuda.is_available() else torch.device("cpu")
    return c
