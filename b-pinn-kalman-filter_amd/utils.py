"""Checkpoint I/O and small helpers (reference utils.py:1-128).

Checkpoint format is the reference's, so checkpoints move both ways:
  score models  {'info': 1, 'optimizer', 'model', 'ema', 'step'}
  PINN          {'info': 0, 'optimizer_1', 'optimizer_2', 'model', 'ema', 'step'}
Score-model state dicts carry the `module.` prefix of the reference's DataParallel
wrapper (models.utils.create_model keeps it).  Loading uses torch.load(weights_only=True):
the files hold only tensors, numbers and containers, so nothing is unpickled beyond data.
"""
from __future__ import annotations

import logging
import os
import time

import torch


class Clock:
    """Prints `info` at most every `itv` seconds (reference utils.py:7-19)."""

    def __init__(self, itv):
        self.itv = itv
        self.start = time.time()

    def tic(self, info: str):
        if time.time() - self.start >= self.itv:
            print(info)
            self.start = time.time()


def show_memory_usage(device):
    print(f"Allocated memory: {torch.cuda.memory_allocated(device) / 1024 ** 2:.2f} MB")
    print(f"Reserved memory: {torch.cuda.memory_reserved(device) / 1024 ** 2:.2f} MB")


def get_ckptdir(workdir, ckpt="checkpoints", ckpt_meta="checkpoints-meta"):
    checkpoint_dir = os.path.join(workdir, ckpt)
    checkpoint_meta_dir = os.path.join(workdir, ckpt_meta, "checkpoint.pth")
    os.makedirs(checkpoint_dir, exist_ok=True)
    os.makedirs(os.path.dirname(checkpoint_meta_dir), exist_ok=True)
    return checkpoint_dir, checkpoint_meta_dir


def _load(path, device):
    return torch.load(path, map_location=device, weights_only=True)


def restore_checkpoint(ckpt_dir, state, device):
    """Resume `state` in place from a checkpoint file; missing file -> state unchanged
    (reference utils.py:39-60, model loaded with strict=False as there)."""
    if not os.path.exists(ckpt_dir):
        os.makedirs(os.path.dirname(ckpt_dir) or ".", exist_ok=True)
        logging.warning(f"No checkpoint found at {ckpt_dir}. Returned the same state as input")
        return state
    loaded = _load(ckpt_dir, device)
    if loaded["info"] == 0:
        state["model"].load_state_dict(loaded["model"], strict=False)
        state["ema"].load_state_dict(loaded["ema"])
        state["step"] = loaded["step"]
        state["optimizer"][0].load_state_dict(loaded["optimizer_1"])
        state["optimizer"][1].load_state_dict(loaded["optimizer_2"])
    else:
        state["optimizer"].load_state_dict(loaded["optimizer"])
        state["model"].load_state_dict(loaded["model"], strict=False)
        state["ema"].load_state_dict(loaded["ema"])
        state["step"] = loaded["step"]
    return state


def load_checkpoint(ckpt_dir, model, device):
    """Model weights only, strict (reference utils.py:98-106)."""
    if not os.path.exists(ckpt_dir):
        logging.warning(f"No checkpoint found at {ckpt_dir}. Returned the same state as input")
        return model
    model.load_state_dict(_load(ckpt_dir, device)["model"])
    return model


def save_checkpoint(ckpt_dir, state):
    if isinstance(state["optimizer"], tuple):
        saved = {"info": 0, "optimizer_1": state["optimizer"][0].state_dict(),
                 "optimizer_2": state["optimizer"][1].state_dict(),
                 "model": state["model"].state_dict(), "ema": state["ema"].state_dict(),
                 "step": state["step"]}
    else:
        saved = {"info": 1, "optimizer": state["optimizer"].state_dict(),
                 "model": state["model"].state_dict(), "ema": state["ema"].state_dict(),
                 "step": state["step"]}
    torch.save(saved, ckpt_dir)
