"""The hipGraph safety gate (op/_hipenv.py): graph replays are trusted only when the HIP runtime
setting DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 provably took effect -- preset in the environment, or
set by `op` before the ROCm runtime of the process started (no /dev/kfd descriptor open yet).
Otherwise get_pinn_step_fn(graph=True) and PCEngine(use_graph=True) run their eager steps, with
one warning.  CPU-only: the late-import case is a subprocess whose runtime "started" first."""
import os
import subprocess
import sys
import warnings

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "b-pinn-kalman-filter_amd")


def _run(code, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k != "DEBUG_CLR_GRAPH_PACKET_CAPTURE"}
    env.update(env_extra or {})
    env["PYTHONPATH"] = os.pathsep.join([PKG, REPO])
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout.strip().splitlines()[-1]


def test_in_process_gate_is_open_here():
    """conftest imports op._hipenv before torch: the setting is proven in effect."""
    from op import _hipenv
    assert os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] == "0"
    assert _hipenv.graph_replays_safe()
    assert _hipenv.graphs_allowed("test")


_PROBE = """
import os, warnings
{pre}
from op import _hipenv
import losses
from configs.pinn import pinn_pde
c = pinn_pde.get_config()
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    g = losses.get_pinn_step_fn(c, train=True, optimize_fn=losses.optimization_manager(c),
                                graph=True)
    g2 = losses.get_pinn_step_fn(c, train=True, optimize_fn=losses.optimization_manager(c),
                                 graph=True)
print(_hipenv.graph_replays_safe(), isinstance(g, losses._PinnGraphStep),
      isinstance(g2, losses._PinnGraphStep), sum("eager step instead" in str(x.message) for x in w))
"""

# the ROCm runtime "started" before `op` is imported: a descriptor of this process whose link
# reads /dev/kfd (here a symlink named so -- the probe reads /proc/self/fd links only)
_STARTED = """
import os, tempfile
d = tempfile.mkdtemp()
link = os.path.join(d, "kfd")
os.symlink("/dev/null", link)
_real = os.readlink
fd = os.open(link, os.O_RDONLY)
os.readlink = lambda p, *a, **k: "/dev/kfd" if p == f"/proc/self/fd/{fd}" else _real(p, *a, **k)
"""


def test_runtime_started_before_import_gets_the_eager_step():
    out = _run(_PROBE.format(pre=_STARTED))
    assert out == "False False False 1", out  # eager both times, warned once


def test_fresh_process_gets_the_graph_step():
    out = _run(_PROBE.format(pre=""))
    assert out == "True True True 0", out


def test_preset_zero_is_trusted_even_after_runtime_start():
    out = _run(_PROBE.format(pre=_STARTED), {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "0"})
    assert out == "True True True 0", out


def test_preset_packet_capture_on_gets_the_eager_step():
    out = _run(_PROBE.format(pre=""), {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "1"})
    assert out == "False False False 1", out


def test_pc_engine_falls_back_to_eager(monkeypatch):
    import torch

    import sampling
    import sde_lib
    from op import _hipenv
    monkeypatch.setattr(_hipenv, "_PROVEN", False)
    monkeypatch.setattr(_hipenv, "_WARNED", set())
    sde = sde_lib.VPSDE(0.1, 20.0, 4)
    with pytest.warns(RuntimeWarning, match="eager step instead"):
        eng = sampling.PCEngine(sde, (1, 1, 4, 4), sampling.EulerMaruyamaPredictor,
                                sampling.LangevinCorrector, 0.075, 1, continuous=True,
                                device=torch.device("cpu"), use_graph=True)
    assert not eng.use_graph
    monkeypatch.setattr(_hipenv, "_PROVEN", True)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        eng = sampling.PCEngine(sde, (1, 1, 4, 4), sampling.EulerMaruyamaPredictor,
                                sampling.LangevinCorrector, 0.075, 1, continuous=True,
                                device=torch.device("cpu"), use_graph=True)
    assert eng.use_graph
