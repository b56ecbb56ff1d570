import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "b-pinn-kalman-filter_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running")


class AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def to_attr(o):
    if isinstance(o, dict):
        return AttrDict({k: to_attr(v) for k, v in o.items()})
    if isinstance(o, list):
        return tuple(to_attr(v) for v in o)
    return o


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name))


def net_fixture(name):
    """(config AttrDict, state dict {key: np.ndarray}, x, labels, y) of tests/golden/net_<name>.npz"""
    d = load_golden(f"net_{name}.npz")
    cfg = to_attr(json.loads(str(d["config_json"])))
    sd = {k[2:]: d[k] for k in d.files if k.startswith("p:")}
    return cfg, sd, d["x"], d["labels"], d["y"]


def product_config(cfg_attr, device):
    """Product ConfigDict built from a fixture config."""
    from configs._configdict import ConfigDict
    c = ConfigDict(json.loads(json.dumps(cfg_attr)))
    c.model.ch_mult = tuple(c.model.ch_mult)
    c.model.attn_resolutions = tuple(c.model.attn_resolutions)
    c.device = device
    return c


@pytest.fixture(scope="session")
def hip():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")
