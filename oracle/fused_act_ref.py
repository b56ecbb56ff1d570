"""ORACLE (test infrastructure only) -- fused bias + leaky-ReLU semantics.

GPU semantics of op/fused_bias_act_kernel.cu:26-47 (slope honoured); the
reference's CPU branch (op/fused_act.py:87-94) hard-codes slope 0.2, which the
fixture tests/golden/fused_lrelu.npz pins.
"""
import numpy as np


def fused_bias_act(x, bias, refer, act, grad, alpha, scale):
    x = np.asarray(x, np.float64)
    if bias is not None and np.size(bias):
        shape = [1] * x.ndim
        shape[1] = -1
        x = x + np.asarray(bias, np.float64).reshape(shape)
    if act == 1:
        y = np.zeros_like(x) if grad == 2 else x
    else:
        if grad == 2:
            y = np.zeros_like(x)
        else:
            mask_src = x if grad == 0 else np.asarray(refer, np.float64)
            y = np.where(mask_src > 0, x, x * alpha)
    return y * scale
