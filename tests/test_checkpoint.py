"""Checkpoint compatibility: the reference's file layout
(utils.py:109-128) round-trips, and a checkpoint written in the reference layout (score
model keys with the DataParallel `module.` prefix) restores into the build's state."""
import torch

from conftest import net_fixture, product_config


def _state(device="cpu"):
    import losses
    import models  # noqa: F401
    from models import utils as mutils
    from models.ema import ExponentialMovingAverage
    cfg, sd, *_ = net_fixture("ddpm_a")
    c = product_config(cfg, torch.device(device))
    c.optim = dict(optimizer="Adam", lr=2e-4, beta1=0.9, eps=1e-8, weight_decay=0, warmup=10,
                   grad_clip=1.0)
    from configs._configdict import ConfigDict
    c.optim = ConfigDict(c.optim)
    model = mutils.create_model(c)            # wrapped: keys carry `module.`
    opt = losses.get_optimizer(c, model.parameters())
    ema = ExponentialMovingAverage(model.parameters(), decay=0.999)
    return dict(optimizer=opt, model=model, ema=ema, step=0), sd


def test_score_checkpoint_round_trip(tmp_path):
    import utils
    state, sd = _state()
    assert all(k.startswith("module.") for k in state["model"].state_dict())
    with torch.no_grad():
        for p in state["model"].parameters():
            p.add_(0.5)
            p.grad = torch.ones_like(p)
    state["optimizer"].step()
    state["ema"].update(state["model"].parameters())
    state["step"] = 17
    path = tmp_path / "checkpoint.pth"
    utils.save_checkpoint(str(path), state)
    raw = torch.load(str(path), weights_only=True)
    assert raw["info"] == 1 and set(raw) == {"info", "optimizer", "model", "ema", "step"}
    fresh, _ = _state()
    utils.restore_checkpoint(str(path), fresh, "cpu")
    assert fresh["step"] == 17
    for (k, a), (_, b) in zip(state["model"].state_dict().items(),
                              fresh["model"].state_dict().items()):
        assert torch.equal(a, b), k
    for a, b in zip(state["ema"].shadow_params, fresh["ema"].shadow_params):
        assert torch.equal(a, b)
    s0 = state["optimizer"].state_dict()["state"]
    s1 = fresh["optimizer"].state_dict()["state"]
    assert all(torch.equal(s0[i]["exp_avg"], s1[i]["exp_avg"]) for i in s0)
    m = _state()[0]["model"]
    utils.load_checkpoint(str(path), m, "cpu")
    assert all(torch.equal(a, b) for a, b in zip(m.state_dict().values(),
                                                 state["model"].state_dict().values()))


def test_reference_layout_weights_load_strict(tmp_path):
    """A file laid out as the reference writes it, with the reference's parameter names
    (tests/golden/net_ddpm_a.npz keys, prefixed `module.` by its DataParallel)."""
    import utils
    state, sd = _state()
    ref_sd = {"module." + k if not k.startswith("module.") else k: torch.tensor(v)
              for k, v in sd.items()}
    path = tmp_path / "ref.pth"
    torch.save({"info": 1, "model": ref_sd, "optimizer": state["optimizer"].state_dict(),
                "ema": state["ema"].state_dict(), "step": 3}, str(path))
    m = _state()[0]["model"]
    utils.load_checkpoint(str(path), m, "cpu")
    for k, v in ref_sd.items():
        assert torch.equal(m.state_dict()[k], v)


def test_pinn_checkpoint_two_optimizers(tmp_path):
    import losses
    import utils
    from configs.pinn import pinn_pde
    from models.ema import ExponentialMovingAverage
    from pinn_kalman.pinn import PINN
    c = pinn_pde.get_config()
    c.device = torch.device("cpu")
    c.model.feature_nums = [4, 8]
    c.data.image_size = 8
    m = PINN(c)
    st = dict(optimizer=(losses.get_optimizer(c, m.flownet.parameters()),
                         losses.get_optimizer(c, m.pressurenet.parameters(), 0.001)),
              model=m, ema=ExponentialMovingAverage(m.parameters(), 0.9), step=5)
    path = tmp_path / "p.pth"
    utils.save_checkpoint(str(path), st)
    assert torch.load(str(path), weights_only=True)["info"] == 0
    m2 = PINN(c)
    st2 = dict(optimizer=(losses.get_optimizer(c, m2.flownet.parameters()),
                          losses.get_optimizer(c, m2.pressurenet.parameters(), 0.001)),
               model=m2, ema=ExponentialMovingAverage(m2.parameters(), 0.9), step=0)
    utils.restore_checkpoint(str(path), st2, "cpu")
    assert st2["step"] == 5
    assert all(torch.equal(a, b) for a, b in zip(m.state_dict().values(), m2.state_dict().values()))
