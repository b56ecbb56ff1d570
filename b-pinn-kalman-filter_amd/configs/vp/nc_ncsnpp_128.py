"""Benchmark config (BASELINE.json configs[2], SURVEY.md 8d cfg #3): NCSN++ hyper-parameters of
configs/vp/cifar10_ncsnpp_continuous.py (its whole model section) on configs/default_nc_configs.py, at 128 x 128 x 1 (nc data), continuous VP-SDE
N = 1000, PC sampler = Euler-Maruyama predictor + Langevin corrector (snr 0.075,
configs/default_nc_configs.py:27), batch 64."""
from configs.default_nc_configs import get_default_configs
from configs.vp import cifar10_ncsnpp_continuous


def get_config():
    c = get_default_configs()
    c.training.update(sde="vpsde", continuous=True, reduce_mean=True, batch_size=64)
    c.sampling.update(method="pc", predictor="euler_maruyama", corrector="langevin", snr=0.075,
                      n_steps_each=1)
    c.data.update(image_size=128, num_channels=1, centered=False)
    c.model.update(cifar10_ncsnpp_continuous.get_config().model)  # the whole model section
    c.model.update(num_scales=1000, dropout=0.)
    return c
