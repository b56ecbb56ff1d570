"""`op.grid_sample.grid_sample_2d` -- bilinear grid sampling, twice differentiable.

Reference: op/grid_sample.py:15-76.  The reference uses ATen for the forward and
first backward and a custom CUDA kernel for the second backward; here all three
are hand-written HIP kernels (csrc/grid_sample.hip).  The autograd structure is
kept: forward -> _GridSample2dBackward (returns grad_input, grad_grid) whose own
backward is the grad2 kernel, so `torch.autograd.grad(..., create_graph=True)`
through `project()` (models/flownet.py:8-25) yields the PINN's second derivatives.
"""
from __future__ import annotations

import torch

from ._lib import check, lib, ptr, require_hip, stream_ptr

_PADDING = {"zeros": 0, "border": 1}


def _fns(dtype):
    if dtype == torch.float32:
        return (lib.bpk_grid_sample2d_fwd_f32, lib.bpk_grid_sample2d_bwd_f32,
                lib.bpk_grid_sample2d_grad2_f32)
    if dtype == torch.float64:
        return (lib.bpk_grid_sample2d_fwd_f64, lib.bpk_grid_sample2d_bwd_f64,
                lib.bpk_grid_sample2d_grad2_f64)
    raise RuntimeError(f"grid_sample_2d: unsupported dtype {dtype}")


def _geom(input, grid):
    N, C, H, W = input.shape
    Ho, Wo = grid.shape[1], grid.shape[2]
    return N, C, H, W, Ho, Wo


def grid_sample2d_fwd_raw(input, grid, padding_mode: int, align_corners: bool):
    require_hip(input, grid, what="grid_sample_2d")
    input, grid = input.contiguous(), grid.contiguous()
    N, C, H, W, Ho, Wo = _geom(input, grid)
    out = torch.empty((N, C, Ho, Wo), device=input.device, dtype=input.dtype)
    check(_fns(input.dtype)[0](input.data_ptr(), grid.data_ptr(), out.data_ptr(), N, C, H, W, Ho,
                               Wo, padding_mode, int(align_corners), stream_ptr(input.device)),
          "grid_sample2d_fwd")
    return out


def grid_sample2d_bwd_raw(grad_out, input, grid, padding_mode, align_corners, need_input=True,
                          need_grid=True):
    grad_out, input, grid = grad_out.contiguous(), input.contiguous(), grid.contiguous()
    N, C, H, W, Ho, Wo = _geom(input, grid)
    gi = torch.zeros_like(input) if need_input else None
    gg = torch.empty_like(grid) if need_grid else None
    check(_fns(input.dtype)[1](grad_out.data_ptr(), input.data_ptr(), grid.data_ptr(),
                               gi.data_ptr() if gi is not None else None,
                               gg.data_ptr() if gg is not None else None, N, C, H, W, Ho, Wo,
                               padding_mode, int(align_corners), stream_ptr(input.device)),
          "grid_sample2d_bwd")
    return gi, gg


def grid_sample2d_grad2_raw(g2_input, g2_grid, grad_out, input, grid, padding_mode,
                            align_corners):
    """g2_input / g2_grid may be None: an all-zero incoming gradient (no fill, no read)."""
    args = [t if t is None else t.contiguous() for t in (g2_input, g2_grid, grad_out, input, grid)]
    g2_input, g2_grid, grad_out, input, grid = args
    N, C, H, W, Ho, Wo = _geom(input, grid)
    ggo = torch.empty_like(grad_out)
    gi = torch.zeros_like(input)
    gg = torch.empty_like(grid)
    check(_fns(input.dtype)[2](ptr(g2_input), ptr(g2_grid), grad_out.data_ptr(),
                               input.data_ptr(), grid.data_ptr(), ggo.data_ptr(), gi.data_ptr(),
                               gg.data_ptr(), N, C, H, W, Ho, Wo, padding_mode, int(align_corners),
                               stream_ptr(input.device)), "grid_sample2d_grad2")
    return ggo, gi, gg


class _GridSample2dForward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, grid, padding_mode="zeros", align_corners=True):
        assert input.ndim == 4 and grid.ndim == 4
        assert input.shape[0] == grid.shape[0] and grid.shape[3] == 2
        pm = _PADDING[padding_mode]
        out = grid_sample2d_fwd_raw(input, grid, pm, align_corners)
        ctx.save_for_backward(input, grid)
        ctx.padding_mode, ctx.align_corners = pm, align_corners
        return out

    @staticmethod
    def backward(ctx, grad_output):
        input, grid = ctx.saved_tensors
        gi, gg = _GridSample2dBackward.apply(grad_output.contiguous(), input, grid,
                                             ctx.padding_mode, ctx.align_corners)
        return gi, gg, None, None


class _GridSample2dBackward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, grad_output, input, grid, padding_mode=0, align_corners=True):
        need_in = ctx.needs_input_grad[1]
        need_grid = ctx.needs_input_grad[2]
        gi, gg = grid_sample2d_bwd_raw(grad_output, input, grid, padding_mode, align_corners,
                                       True, True)
        ctx.save_for_backward(grad_output, input, grid)
        ctx.padding_mode, ctx.align_corners = padding_mode, align_corners
        del need_in, need_grid
        return gi, gg

    @staticmethod
    def backward(ctx, g2_input, g2_grid):
        grad_output, input, grid = ctx.saved_tensors
        # a None incoming gradient goes to the kernel as NULL (all zero)
        ggo, gi, gg = grid_sample2d_grad2_raw(g2_input, g2_grid, grad_output, input, grid,
                                              ctx.padding_mode, ctx.align_corners)
        return ggo, gi, gg, None, None


def grid_sample_2d(input, grid, padding_mode="zeros", align_corners=True):
    assert padding_mode in ["zeros", "border"]
    require_hip(input, grid, what="grid_sample_2d")
    # The callers' grids are NHWC views of NCHW tensors (flownet.project): made dense once
    # here, as a recorded (differentiable) copy, so the Functions save dense tensors that are
    # not copied again by each backward / double backward.  The copy must stay OUTSIDE the
    # Functions: a tensor made inside forward and saved is cut from the graph, and the
    # double backward's grad_grid / grad_input (the PINN residual's second-order terms
    # through the warp) would silently vanish -- likewise grad_output above.
    return _GridSample2dForward.apply(input.contiguous(), grid.contiguous(), padding_mode,
                                      align_corners)


def _fns3(dtype):
    if dtype == torch.float32:
        return (lib.bpk_grid_sample3d_fwd_f32, lib.bpk_grid_sample3d_bwd_f32,
                lib.bpk_grid_sample3d_grad2_f32)
    if dtype == torch.float64:
        return (lib.bpk_grid_sample3d_fwd_f64, lib.bpk_grid_sample3d_bwd_f64,
                lib.bpk_grid_sample3d_grad2_f64)
    raise RuntimeError(f"grid_sample_3d: unsupported dtype {dtype}")


def _geom3(input, grid):
    N, C, D, H, W = input.shape
    return N, C, D, H, W, grid.shape[1], grid.shape[2], grid.shape[3]


def grid_sample3d_fwd_raw(input, grid, padding_mode: int, align_corners: bool):
    require_hip(input, grid, what="grid_sample_3d")
    input, grid = input.contiguous(), grid.contiguous()
    N, C, D, H, W, Do, Ho, Wo = _geom3(input, grid)
    out = torch.empty((N, C, Do, Ho, Wo), device=input.device, dtype=input.dtype)
    check(_fns3(input.dtype)[0](input.data_ptr(), grid.data_ptr(), out.data_ptr(), N, C, D, H, W,
                                Do, Ho, Wo, padding_mode, int(align_corners),
                                stream_ptr(input.device)), "grid_sample3d_fwd")
    return out


def grid_sample3d_bwd_raw(grad_out, input, grid, padding_mode, align_corners):
    grad_out, input, grid = grad_out.contiguous(), input.contiguous(), grid.contiguous()
    N, C, D, H, W, Do, Ho, Wo = _geom3(input, grid)
    gi = torch.zeros_like(input)
    gg = torch.empty_like(grid)
    check(_fns3(input.dtype)[1](grad_out.data_ptr(), input.data_ptr(), grid.data_ptr(),
                                gi.data_ptr(), gg.data_ptr(), N, C, D, H, W, Do, Ho, Wo,
                                padding_mode, int(align_corners), stream_ptr(input.device)),
          "grid_sample3d_bwd")
    return gi, gg


def grid_sample3d_grad2_raw(g2_input, g2_grid, grad_out, input, grid, padding_mode,
                            align_corners):
    g2_input, g2_grid, grad_out, input, grid = (
        t.contiguous() for t in (g2_input, g2_grid, grad_out, input, grid))
    N, C, D, H, W, Do, Ho, Wo = _geom3(input, grid)
    ggo = torch.empty_like(grad_out)
    gi = torch.zeros_like(input)
    gg = torch.empty_like(grid)
    check(_fns3(input.dtype)[2](g2_input.data_ptr(), g2_grid.data_ptr(), grad_out.data_ptr(),
                                input.data_ptr(), grid.data_ptr(), ggo.data_ptr(), gi.data_ptr(),
                                gg.data_ptr(), N, C, D, H, W, Do, Ho, Wo, padding_mode,
                                int(align_corners), stream_ptr(input.device)),
          "grid_sample3d_grad2")
    return ggo, gi, gg


class _GridSample3dForward(torch.autograd.Function):
    """reference op/grid_sample.py:79-99"""

    @staticmethod
    def forward(ctx, input, grid, padding_mode="zeros", align_corners=True):
        assert input.ndim == 5 and grid.ndim == 5
        assert input.shape[0] == grid.shape[0] and grid.shape[4] == 3
        pm = _PADDING[padding_mode]
        out = grid_sample3d_fwd_raw(input, grid, pm, align_corners)
        ctx.save_for_backward(input, grid)
        ctx.padding_mode, ctx.align_corners = pm, align_corners
        return out

    @staticmethod
    def backward(ctx, grad_output):
        input, grid = ctx.saved_tensors
        gi, gg = _GridSample3dBackward.apply(grad_output, input, grid, ctx.padding_mode,
                                             ctx.align_corners)
        return gi, gg, None, None


class _GridSample3dBackward(torch.autograd.Function):
    """reference op/grid_sample.py:102-131: first backward (aten::grid_sampler_3d_backward
    there), whose own backward is the double-backward kernel (grad2_3d)"""

    @staticmethod
    def forward(ctx, grad_output, input, grid, padding_mode=0, align_corners=True):
        gi, gg = grid_sample3d_bwd_raw(grad_output, input, grid, padding_mode, align_corners)
        ctx.save_for_backward(grad_output, input, grid)
        ctx.padding_mode, ctx.align_corners = padding_mode, align_corners
        return gi, gg

    @staticmethod
    def backward(ctx, g2_input, g2_grid):
        grad_output, input, grid = ctx.saved_tensors
        if g2_input is None:
            g2_input = torch.zeros_like(input)
        if g2_grid is None:
            g2_grid = torch.zeros_like(grid)
        ggo, gi, gg = grid_sample3d_grad2_raw(g2_input, g2_grid, grad_output, input, grid,
                                              ctx.padding_mode, ctx.align_corners)
        return ggo, gi, gg, None, None


def grid_sample_3d(input, grid, padding_mode="zeros", align_corners=True):
    """Trilinear grid sampling of [N, C, D, H, W] at grid [N, Do, Ho, Wo, 3] (x, y, z),
    twice differentiable (reference op/grid_sample.py:19-22; no caller on the hot path)."""
    assert padding_mode in ["zeros", "border"]
    require_hip(input, grid, what="grid_sample_3d")
    return _GridSample3dForward.apply(input, grid, padding_mode, align_corners)
