"""Dispatcher registration of the reference's extension entry points over the C ABI.

The reference's pybind extensions are reachable as `upfirdn2d_op.upfirdn2d(...)`,
`fused.fused_bias_act(...)`, `gridsample_grad2.grad2_2d / grad2_3d(...)` and
`ns_step_forward.update_{density,velocity,pressure}(...)` (op/upfirdn2d.cpp:12-22,
op/fused_bias_act.cpp:11-20, op/grid_sample.cpp:26-57, op/ns_step.cpp:45-107).  The same
names and argument lists are registered here as torch.library operators, so they appear
in `torch.ops.<extension>.<name>` and go through the dispatcher (CUDA = HIP key; no CPU
kernel, so a CPU tensor fails loudly), with fake (meta) kernels for shape propagation.
Each body is one call into libbpk.so -- the same call the op/* wrappers make.

The op/* wrappers themselves keep calling the C ABI directly from their autograd
Functions: a dispatcher round trip costs ~10-20 us of host time per call, and the
PINN step (15 k launches) is host-bound.
"""
from __future__ import annotations

from typing import List

import torch
from torch.library import custom_op

from . import correlation as _corr
from . import grid_sample as _gs
from . import ns_step as _ns
from ._lib import check, lib, require_hip, stream_ptr
from .fused_act import fused_bias_act_raw

Tensor = torch.Tensor


def _up_out(in_h, in_w, kh, kw, up_x, up_y, down_x, down_y, px0, px1, py0, py1):
    return (in_h * up_y + py0 + py1 - kh) // down_y + 1, (in_w * up_x + px0 + px1 - kw) // down_x + 1


@custom_op("upfirdn2d_op::upfirdn2d", mutates_args=(), device_types="cuda")
def upfirdn2d_op(input: Tensor, kernel: Tensor, up_x: int, up_y: int, down_x: int, down_y: int,
                 pad_x0: int, pad_x1: int, pad_y0: int, pad_y1: int) -> Tensor:
    """input [major, in_h, in_w, minor] (the reference extension's layout), kernel [kh, kw]."""
    require_hip(input, kernel, what="upfirdn2d_op.upfirdn2d")
    x = input.contiguous()
    k = kernel.to(device=x.device, dtype=x.dtype).contiguous()
    major, in_h, in_w, minor = x.shape
    kh, kw = k.shape
    out_h, out_w = _up_out(in_h, in_w, kh, kw, up_x, up_y, down_x, down_y, pad_x0, pad_x1,
                           pad_y0, pad_y1)
    out = x.new_empty((major, out_h, out_w, minor))
    fn = lib.bpk_upfirdn2d_f32 if x.dtype == torch.float32 else lib.bpk_upfirdn2d_f64
    check(fn(x.data_ptr(), k.data_ptr(), out.data_ptr(), major, in_h, in_w, minor, kh, kw, up_x,
             up_y, down_x, down_y, pad_x0, pad_x1, pad_y0, pad_y1, out_h, out_w,
             stream_ptr(x.device)), "upfirdn2d_op.upfirdn2d")
    return out


@upfirdn2d_op.register_fake
def _(input, kernel, up_x, up_y, down_x, down_y, pad_x0, pad_x1, pad_y0, pad_y1):
    major, in_h, in_w, minor = input.shape
    out_h, out_w = _up_out(in_h, in_w, kernel.shape[0], kernel.shape[1], up_x, up_y, down_x,
                           down_y, pad_x0, pad_x1, pad_y0, pad_y1)
    return input.new_empty((major, out_h, out_w, minor))


@custom_op("fused::fused_bias_act", mutates_args=(), device_types="cuda")
def fused_bias_act(input: Tensor, bias: Tensor, refer: Tensor, act: int, grad: int, alpha: float,
                   scale: float) -> Tensor:
    return fused_bias_act_raw(input, bias, refer, act, grad, alpha, scale)


@fused_bias_act.register_fake
def _(input, bias, refer, act, grad, alpha, scale):
    return torch.empty_like(input)


@custom_op("gridsample_grad2::grad2_2d", mutates_args=(), device_types="cuda")
def grad2_2d(grad2_grad_input: Tensor, grad2_grad_grid: Tensor, grad_output: Tensor, input: Tensor,
             grid: Tensor, padding_mode: bool, align_corners: bool) -> List[Tensor]:
    return list(_gs.grid_sample2d_grad2_raw(grad2_grad_input, grad2_grad_grid, grad_output, input,
                                            grid, int(padding_mode), align_corners))


@grad2_2d.register_fake
def _(grad2_grad_input, grad2_grad_grid, grad_output, input, grid, padding_mode, align_corners):
    return [torch.empty_like(grad_output), torch.empty_like(input), torch.empty_like(grid)]


@custom_op("gridsample_grad2::grad2_3d", mutates_args=(), device_types="cuda")
def grad2_3d(grad2_grad_input: Tensor, grad2_grad_grid: Tensor, grad_output: Tensor, input: Tensor,
             grid: Tensor, padding_mode: bool, align_corners: bool) -> List[Tensor]:
    return list(_gs.grid_sample3d_grad2_raw(grad2_grad_input, grad2_grad_grid, grad_output, input,
                                            grid, int(padding_mode), align_corners))


@grad2_3d.register_fake
def _(grad2_grad_input, grad2_grad_grid, grad_output, input, grid, padding_mode, align_corners):
    return [torch.empty_like(grad_output), torch.empty_like(input), torch.empty_like(grid)]


@custom_op("ns_step_forward::update_density", mutates_args=(), device_types="cuda")
def update_density(dens: Tensor, vel: Tensor, dt: float, dx: float) -> Tensor:
    return _ns.update_density(dens, vel, dt, dx)


@custom_op("ns_step_forward::update_velocity", mutates_args=(), device_types="cuda")
def update_velocity(vel: Tensor, pres: Tensor, dt: float, dx: float) -> Tensor:
    return _ns.update_velocity(vel, pres, dt, dx)


@custom_op("ns_step_forward::update_pressure", mutates_args=(), device_types="cuda")
def update_pressure(pres: Tensor, vel: Tensor, dt: float, dx: float) -> Tensor:
    return _ns.update_pressure(pres, vel, dt, dx)


for _op in (update_density, update_velocity, update_pressure):
    _op.register_fake(lambda a, b, dt, dx: torch.empty_like(a))


@custom_op("correlation::forward", mutates_args=(), device_types="cuda")
def correlation_forward(first: Tensor, second: Tensor, stride: int) -> Tensor:
    """The CuPy kernel_Correlation_updateOutput of op/correlation.py:34-102 (no extension
    there; the name follows the module)."""
    require_hip(first, second, what="correlation.forward")
    return _corr.correlation_fwd_raw(first.contiguous(), second.contiguous(), stride)


@correlation_forward.register_fake
def _(first, second, stride):
    B, C, H, W = first.shape
    return first.new_empty((B, 49, -(-H // stride), -(-W // stride)))
