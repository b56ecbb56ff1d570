"""CPU: the C-ABI library builds/loads and exports every entry point of include/bpk.h."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import REPO


def test_header_parses_and_library_exports_every_symbol():
    from op import _lib
    protos = _lib.parse_header()
    assert len(protos) >= 30
    assert os.path.exists(_lib.LIB_PATH), "build libbpk.so first (__graft_entry__.build())"
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = set(re.findall(r" T (bpk_\w+)", out))
    missing = sorted(set(protos) - exported)
    assert not missing, f"declared in bpk.h but not exported: {missing}"


def test_library_loads_and_reports_abi_version():
    from op import _lib
    dll = _lib.lib.load()
    assert dll.bpk_abi_version() == 1
    assert dll.bpk_last_error() is not None


def test_argument_errors_are_reported_without_a_device():
    """Argument validation happens before any HIP call, so it works on a GPU-less host."""
    from op import _lib
    dll = _lib.lib.load()
    rc = dll.bpk_upfirdn2d_f32(None, None, None, 1, 4, 4, 1, 4, 4, 1, 1, 2, 2, 1, 1, 1, 1,
                               99, 99, None)  # wrong out shape
    assert rc == 1
    assert b"out shape" in dll.bpk_last_error()
    rc = dll.bpk_ns_update_velocity_f32(None, None, None, None, 2, 1, 5, 0.1, 0.1, 1, None)
    assert rc == 1 and b"planes" in dll.bpk_last_error()
    rc = dll.bpk_group_norm_fwd_f32(None, None, None, None, None, None, None, None, 2, 30, 16, 32,
                                    1e-6, 1, None)
    assert rc == 1 and b"divisible" in dll.bpk_last_error()
    with pytest.raises(RuntimeError, match="status 1"):
        _lib.check(1, "probe")


def test_workspace_queries():
    from op import _lib
    dll = _lib.lib.load()
    assert dll.bpk_ns_workspace_bytes(1, 4, 8, 8) == 8 * 4 * 64 * 4
    assert dll.bpk_group_norm_workspace_bytes(2, 64, 128 * 128, 32) > 0
    assert dll.bpk_langevin_workspace_bytes(64, 128 * 128) == 64 * 4 * 2 * 4


def test_product_ops_refuse_cpu_tensors():
    """No silent CPU fallback: the product op path raises on host tensors."""
    import torch
    from op import upfirdn2d, ns_step
    from op.norm_act import group_norm_act
    x = torch.zeros(1, 1, 8, 8)
    with pytest.raises(RuntimeError, match="HIP"):
        upfirdn2d(x, torch.ones(2, 2) / 4, down=2)
    with pytest.raises(RuntimeError, match="HIP"):
        ns_step.update_pressure(x, torch.zeros(1, 2, 8, 8), 0.1, 0.1)
    with pytest.raises(RuntimeError, match="HIP"):
        group_norm_act(torch.zeros(1, 4, 4, 4), torch.nn.GroupNorm(2, 4))


def test_reference_extension_names_are_dispatcher_ops():
    """torch.ops.<extension>.<name> exist for every reference pybind entry point
    (op/upfirdn2d.cpp:12-22, op/fused_bias_act.cpp:11-20, op/grid_sample.cpp:26-57,
    op/ns_step.cpp:45-107), with no CPU kernel: a CPU tensor fails loudly."""
    import pytest
    import torch
    import op  # noqa: F401
    names = [("upfirdn2d_op", "upfirdn2d"), ("fused", "fused_bias_act"),
             ("gridsample_grad2", "grad2_2d"), ("gridsample_grad2", "grad2_3d"),
             ("ns_step_forward", "update_density"), ("ns_step_forward", "update_velocity"),
             ("ns_step_forward", "update_pressure"), ("correlation", "forward")]
    for ns, name in names:
        assert hasattr(getattr(torch.ops, ns), name), (ns, name)
    with pytest.raises((NotImplementedError, RuntimeError)):
        torch.ops.upfirdn2d_op.upfirdn2d(torch.zeros(1, 4, 4, 1), torch.ones(2, 2), 1, 1, 1, 1,
                                         0, 0, 0, 0)
