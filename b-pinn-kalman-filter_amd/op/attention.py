"""Fused self-attention of the score networks' attention blocks at inference (csrc/attention.hip).

`attention(qkv, scale)` == bmm(v, softmax(scale * bmm(q^T, k), -1)^T) for qkv [B, 3, C, P]
(q, k, v the three channel blocks of the stacked NIN_0/1/2 projection, P = H*W), returning
[B, C, P]: what AttnBlockpp (reference models/layerspp.py:75-91) and AttnBlock
(models/layers.py:549-573) compute between their projections, with the [P, P] logits kept
on chip.  Inference only (no autograd); HIP tensors only.
"""
from __future__ import annotations

import torch

from ._lib import check, lib, require_hip, stream_ptr


def supported(qkv) -> bool:
    if qkv.dim() != 4 or qkv.shape[1] != 3 or qkv.dtype != torch.float32 or not qkv.is_cuda:
        return False
    B, _, C, P = qkv.shape
    return bool(lib.bpk_attention_supported(B, C, P))


def attention(qkv, scale):
    require_hip(qkv, what="attention")
    if not supported(qkv):
        raise RuntimeError(f"attention: unsupported qkv {tuple(qkv.shape)} {qkv.dtype}")
    qkv = qkv.detach().contiguous()
    B, _, C, P = qkv.shape
    out = torch.empty((B, C, P), dtype=torch.float32, device=qkv.device)
    # key splits (partials + a combine launch) when the batch is too small to fill the chip
    nws = lib.bpk_attention_workspace_bytes(B, C, P)
    ws = torch.empty(nws // 4, dtype=torch.float32, device=qkv.device) if nws > 0 else None
    check(lib.bpk_attention_ex_f32(qkv.data_ptr(), out.data_ptr(),
                                   None if ws is None else ws.data_ptr(), B, C, P, float(scale),
                                   stream_ptr(qkv.device)), "attention")
    return out
