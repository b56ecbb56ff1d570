"""CPU checks of the build's config modules and networks against the reference's, as
recorded in the config-level fixtures (tests/golden/make_golden_configs.py): every key of
the reference config has the same value in the build's config (after the same test
overrides), and the build's network has exactly the reference's parameters and shapes
(the seeded weights of the GPU parity tests are keyed by those names)."""
import importlib
import json

import pytest
import torch

from conftest import full_pinn_config, load_golden

CASES = [  # fixture, build config module, overrides applied on both sides
    ("cfg_ddpmpp_cifar.npz", "configs.vp.cifar10_ddpmpp_continuous", {"model.dropout": 0.0}),
    ("cfg_ncsnpp_cifar.npz", "configs.vp.cifar10_ncsnpp_continuous", {"model.dropout": 0.0}),
    ("cfg_ncsnpp128_pc.npz", "configs.vp.nc_ncsnpp_128", {}),
    ("cfg_ncddpmpp128_pc.npz", "configs.vp.nc_ddpmpp", {"data.image_size": 128}),
    ("cfg_dps256.npz", "configs.inverse.nc_ddpmpp_inpaint_dps", {"data.image_size": 256}),
]
SECTIONS = ("training", "sampling", "data", "model", "optim", "inverse")


def _cfg(module, overrides):
    c = importlib.import_module(module).get_config()
    for k, v in overrides.items():
        sec, key = k.split(".")
        c[sec][key] = v
    c.device = torch.device("cpu")
    return c


def _plain(v):
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    if isinstance(v, (tuple, list)):
        return [_plain(x) for x in v]
    return v


def _compare(ref, mine, path=""):
    bad = []
    for k, v in ref.items():
        if k == "device":
            continue
        if k not in mine:
            bad.append(f"{path}{k}: missing")
        elif isinstance(v, dict):
            bad += _compare(v, mine[k], f"{path}{k}.")
        elif _plain(mine[k]) != v:
            bad.append(f"{path}{k}: reference {v!r}, build {_plain(mine[k])!r}")
    return bad


def _check_config(ref_json, c, skip=()):
    ref = json.loads(ref_json)
    bad = []
    for sec in SECTIONS:
        if sec in ref and sec not in skip:
            bad += _compare(ref[sec], c[sec], sec + ".")
    assert not bad, "\n".join(bad)


def _check_params(shapes_json, model):
    ref = json.loads(shapes_json)
    mine = {k: list(p.shape) for k, p in model.named_parameters()}
    assert mine == ref


@pytest.mark.parametrize("fixture,module,overrides", CASES)
def test_score_configs_and_networks_match_reference(fixture, module, overrides):
    import models  # noqa: F401
    from models import utils as mutils
    d = load_golden(fixture)
    ref = json.loads(str(d["config_json"]))
    c = _cfg(module, overrides)
    # data-set bookkeeping the build does not read (paths, categories) is not compared
    _check_config(str(d["config_json"]), c)
    assert ref["model"]["name"] == c.model.name
    _check_params(str(d["param_shapes"]), mutils.create_model(c, wrap=False))


def test_pinn_config_and_network_match_reference():
    from configs.pinn import pinn_pde
    from pinn_kalman.pinn import PINN
    d = load_golden("cfg_pinn64.npz")
    c = full_pinn_config(pinn_pde.get_config)
    _check_config(str(d["config_json"]), c)
    _check_params(str(d["param_shapes"]), PINN(c))
