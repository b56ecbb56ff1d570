"""Exponential moving average of parameters (reference: models/ema.py:10-97).

Same API (`update`, `copy_to`, `store`, `restore`, `state_dict`,
`load_state_dict`) and decay schedule min(decay, (1 + n) / (10 + n)).  The
update is one multi-tensor `torch._foreach_lerp_` launch set over all shadow
parameters instead of a Python loop of per-tensor kernels:
    s <- s - (1 - d) (s - p)  ==  lerp(s, p, 1 - d).
"""
from __future__ import annotations

import torch


class ExponentialMovingAverage:
    def __init__(self, parameters, decay, use_num_updates=True):
        if decay < 0.0 or decay > 1.0:
            raise ValueError("Decay must be between 0 and 1")
        self.decay = decay
        self.num_updates = 0 if use_num_updates else None
        self.shadow_params = [p.clone().detach() for p in parameters if p.requires_grad]
        self.collected_params = []

    def update(self, parameters):
        decay = self.decay
        if self.num_updates is not None:
            self.num_updates += 1
            decay = min(decay, (1 + self.num_updates) / (10 + self.num_updates))
        with torch.no_grad():
            params = [p for p in parameters if p.requires_grad]
            torch._foreach_lerp_(self.shadow_params, params, 1.0 - decay)

    def copy_to(self, parameters):
        # In-place copies under no_grad (not `p.data.copy_`): they bump the parameter's
        # version counter, which keys the cached Winograd filter transforms (op/conv.py).
        params = [p for p in parameters if p.requires_grad]
        with torch.no_grad():
            for s, p in zip(self.shadow_params, params):
                p.copy_(s)

    def store(self, parameters):
        self.collected_params = [p.detach().clone() for p in parameters]

    def restore(self, parameters):
        with torch.no_grad():
            for c, p in zip(self.collected_params, parameters):
                p.copy_(c)

    def state_dict(self):
        return dict(decay=self.decay, num_updates=self.num_updates,
                    shadow_params=self.shadow_params)

    def load_state_dict(self, state_dict):
        self.decay = state_dict["decay"]
        self.num_updates = state_dict["num_updates"]
        self.shadow_params = state_dict["shadow_params"]
