"""Inpainting measurement operator in gather form (reference inverse/operators.py:8-205).

`InpaintOperator(mask=<iterable of masks>)`: `next()` advances to the next mask
(cycling, reference :134-142); `op(x, keep_shape=True)` = mask * x, and
`keep_shape=False` returns the observed pixels [B, C, K] -- what the reference
computes as `bcmm(pL, x)` with a dense [N, 1, HW, K] selection matrix (:125-130,
:186-197).  Here the selection is an index gather: no HW x HW matrices (which the
reference builds in `__init__` and which do not fit at 256^2).

`random_mask_source(config)` replaces `datasets.get_mask_dataset` for
operator='inpaint_rnd' (reference datasets.py:290-300): per-pixel uniform noise
thresholded at `ratio` (kept where u <= ratio when invert=False, Binarize
datasets.py:41-51), one mask repeated across the batch (Repeat :54-60).
"""
from __future__ import annotations

import torch


def random_mask_source(config, n=1600, generator=None):
    """List of [B, 1, H, W] float masks (synthetic; the reference draws torch.rand too)."""
    size = config.data.image_size
    u = torch.rand(n, size, size, generator=generator)
    keep = u > config.inverse.ratio
    if not config.inverse.invert:
        keep = ~keep
    m = keep.float()
    B = config.training.batch_size
    return [m[i].expand(B, 1, size, size).contiguous() for i in range(n)]


def get_operator(config, mask_source=None):
    if config.inverse.operator not in ("inpaint", "inpaint_rnd"):
        raise NotImplementedError(config.inverse.operator)
    if mask_source is None:
        mask_source = random_mask_source(config)
    return InpaintOperator(mask=mask_source)


class InpaintOperator:
    def __init__(self, **kwargs):
        self.params = kwargs
        self.iter = None
        self.mask = None
        self.next()

    def next(self):
        if self.iter is None:
            self.iter = iter(self.params["mask"])
        try:
            self.mask = next(self.iter)
        except StopIteration:
            self.iter = iter(self.params["mask"])
            self.mask = next(self.iter)
        self._idx = None

    def _observed(self, invert):
        """[B, K] observed-pixel indices of the current mask, computed once per mask (the
        nonzero / count check syncs with the host; the DPS drift applies the operator at
        every function evaluation with the same mask)."""
        key = (invert, id(self.mask), self.mask._version, self.mask.device)
        if self._idx is not None and self._idx[0] == key:
            return self._idx[1]
        m = (1 - self.mask) if invert else self.mask
        # one index list per sample; the reference's torch.stack needs equal counts
        flat = m.reshape(m.shape[0], -1)
        idx = [torch.nonzero(row > 0.5, as_tuple=False).squeeze(1) for row in flat]
        if len({int(i.numel()) for i in idx}) != 1:
            raise ValueError("inpaint operator: samples observe different pixel counts")
        idx = torch.stack(idx)
        self._idx = (key, idx, self.mask)  # the mask is kept alive with its key
        return idx

    def __call__(self, x, keep_shape=True, invert=False):
        assert self.mask.shape == x.shape, (self.mask.shape, x.shape)
        if self.mask.device != x.device:
            self.mask = self.mask.to(x.device)
        if keep_shape:
            return (1 - self.mask) * x if invert else self.mask * x
        idx = self._observed(invert)                          # [B, K]
        B, C = x.shape[:2]
        flat = x.reshape(B, C, -1)
        return torch.gather(flat, 2, idx[:, None, :].expand(B, C, idx.shape[1]))

    def transpose(self, y, shape, invert=False):
        """A^T y: scatter observed values back to [B, C, H, W] (zeros elsewhere)."""
        idx = self._observed(invert).to(y.device)
        B, C = shape[:2]
        out = y.new_zeros(B, C, shape[2] * shape[3])
        out.scatter_(2, idx[:, None, :].expand(B, C, idx.shape[1]), y)
        return out.view(shape)
