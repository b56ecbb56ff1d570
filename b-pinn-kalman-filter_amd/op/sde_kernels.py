"""Thin wrappers over the PC-sampler kernels of csrc/sampler.hip (see include/bpk.h).

All tensors are float32 on the HIP device.  `coef` is a [n_rows, coef_bdim, 8]
table (or [coef_bdim, 8] for a single step), `step` a 1-element int32 device
tensor holding the row index (so captured graphs can advance it on device).
"""
from __future__ import annotations

import torch

from ._lib import check, lib, require_hip, stream_ptr

COEF_STRIDE = 8
C_SDIV, C_DRIFT, C_DIFF, C_DT, C_SQRT_MDT, C_ALPHA, C_AUX = range(7)

PRED_EM, PRED_RD, PRED_ANC_VP, PRED_ANC_VE = 0, 1, 2, 3
SCORE_DIV, SCORE_RAW = 0, 1


def _p(t):
    return None if t is None else t.data_ptr()


def _bd(coef, B):
    bdim = coef.shape[-2]
    if bdim not in (1, B):
        raise RuntimeError(f"coef table batch dim {bdim} must be 1 or {B}")
    return bdim


def philox_normal(shape, seed, step, draw, sample_offset=0, device=None):
    out = torch.empty(shape, device=device, dtype=torch.float32)
    B = shape[0]
    D = out.numel() // max(B, 1)
    check(lib.bpk_philox_normal_f32(out.data_ptr(), B, D, sample_offset, seed & (2 ** 64 - 1),
                                    _p(step), draw, stream_ptr(out.device)), "philox_normal")
    return out


def predictor(kind, x, model_out, coef, step, *, x_out, x_mean=None, noise=None, score_mode=0,
              drift_mul_x=1, seed=0, draw=0, sample_offset=0):
    require_hip(x, model_out, coef, step, what="pc_predictor")
    B = x.shape[0]
    D = x.numel() // B
    check(lib.bpk_pc_predictor_f32(kind, x.data_ptr(), model_out.data_ptr(), _p(noise),
                                   x_out.data_ptr(), _p(x_mean), B, D, sample_offset,
                                   coef.data_ptr(), _bd(coef, B), step.data_ptr(), score_mode,
                                   drift_mul_x, seed & (2 ** 64 - 1), draw,
                                   stream_ptr(x.device)), "pc_predictor")


def langevin_workspace(B, D, device):
    nb = lib.bpk_langevin_workspace_bytes(B, D)
    return torch.empty(max(nb // 4, 1), device=device, dtype=torch.float32)


def langevin_norms(model_out, coef, step, workspace, red, *, noise=None, score_mode=0, seed=0,
                   draw=0, sample_offset=0):
    """red[0] = sum_b ||score_b||, red[1] = sum_b ||noise_b|| over the local batch."""
    B = model_out.shape[0]
    D = model_out.numel() // B
    st = stream_ptr(model_out.device)
    check(lib.bpk_langevin_partial_f32(model_out.data_ptr(), _p(noise), workspace.data_ptr(), B, D,
                                       sample_offset, coef.data_ptr(), _bd(coef, B),
                                       step.data_ptr(), score_mode, seed & (2 ** 64 - 1), draw,
                                       st), "langevin_partial")
    check(lib.bpk_langevin_reduce_f32(workspace.data_ptr(), red.data_ptr(), B, D, st),
          "langevin_reduce")


def langevin_update(mode, x, model_out, coef, step, red, *, x_out, x_mean=None, noise=None,
                    B_global=None, score_mode=0, snr=0.16, seed=0, draw=0, sample_offset=0):
    B = x.shape[0]
    D = x.numel() // B
    check(lib.bpk_langevin_update_f32(mode, x.data_ptr(), model_out.data_ptr(), _p(noise),
                                      _p(red), x_out.data_ptr(), _p(x_mean), B, D,
                                      B_global or B, sample_offset, coef.data_ptr(),
                                      _bd(coef, B), step.data_ptr(), score_mode, float(snr),
                                      seed & (2 ** 64 - 1), draw, stream_ptr(x.device)),
          "langevin_update")


def step_increment(step):
    check(lib.bpk_step_increment(step.data_ptr(), stream_ptr(step.device)), "step_increment")


def fill_from_table(out, table, step):
    check(lib.bpk_fill_step_scalar_f32(out.data_ptr(), out.numel(), table.data_ptr(),
                                       step.data_ptr(), stream_ptr(out.device)),
          "fill_step_scalar")
