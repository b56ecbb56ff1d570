"""Native ops of the hot path on hand-written gfx950 HIP kernels.

Mirrors the reference package `op/` (op/__init__.py:1-2): `upfirdn2d`,
`fused_leaky_relu` / `FusedLeakyReLU`, and the submodules `grid_sample` and
`ns_step`, `correlation`; plus the build's fused block ops (`norm_act`) and PC-sampler kernels
(`sde_kernels`).  All of them call libbpk.so through the C ABI of include/bpk.h; the
reference's extension entry points are also registered with the dispatcher (`torch_ops`).
"""
from . import _hipenv  # noqa: F401  (HIP runtime settings: before any device call)
from .fused_act import FusedLeakyReLU, fused_leaky_relu
from .upfirdn2d import upfirdn2d
from . import correlation, grid_sample, ns_step, norm_act, sde_kernels
from . import torch_ops  # torch.ops.{upfirdn2d_op, fused, gridsample_grad2, ns_step_forward}

__all__ = ["FusedLeakyReLU", "fused_leaky_relu", "upfirdn2d", "correlation", "grid_sample", "ns_step",
           "norm_act", "sde_kernels"]
