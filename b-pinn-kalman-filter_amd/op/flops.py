"""FLOP tally of one measured step (bench.py's roofline objects; measurement only).

The native MFMA kernels are launched through ctypes, which torch's FlopCounterMode cannot
see, so every launch site in op/conv.py reports its own count here while a `counting()`
block is open; the aten ops that remain (MIOpen convolutions the per-call selection keeps,
rocBLAS bmm of the attention blocks, linear layers) are counted inside the same block by a
TorchDispatchMode over torch.utils.flop_counter's per-op formulas (FlopCounterMode itself
adds module-tracking autograd hooks that cannot run inside the PINN residual's
torch.autograd.grad passes).  Two bases per launch:
  executed  the multiplies the kernel actually issues -- Winograd F(2x2,3x3) does 16 per
            2x2 output tile per (cin, cout), i.e. 4/9 of the direct count;
  direct    2 * MACs of the direct convolution / GEMM (SURVEY.md 8(d)'s FlopCounterMode basis).
aten ops are counted on the direct basis in both (what MIOpen executes is not visible).
Outside a `counting()` block `add` is one list check.
"""
from __future__ import annotations

import contextlib

_ACTIVE: list = []


class Tally:
    def __init__(self):
        self.executed = 0.0
        self.direct = 0.0
        self.by_kind: dict = {}
        self.aten = 0.0

    def add(self, kind, executed, direct):
        self.executed += executed
        self.direct += direct
        e, d, n = self.by_kind.get(kind, (0.0, 0.0, 0))
        self.by_kind[kind] = (e + executed, d + direct, n + 1)

    @property
    def total_executed(self):
        return self.executed + self.aten

    @property
    def total_direct(self):
        return self.direct + self.aten

    def summary(self):
        return {"executed_flop": self.total_executed, "direct_flop": self.total_direct,
                "aten_flop": self.aten,
                "native": {k: {"executed": e, "direct": d, "launches": n}
                           for k, (e, d, n) in sorted(self.by_kind.items())}}


def add(kind, executed, direct=None):
    if _ACTIVE:
        for t in _ACTIVE:
            t.add(kind, float(executed), float(executed if direct is None else direct))


def wino3x3(kind, N, C, Cout, H, W):
    """Winograd F(2x2,3x3): 16 multiplies per 2x2 tile per (cin, cout) vs 9 per pixel."""
    if _ACTIVE:
        add(kind, 32.0 * N * C * Cout * ((H + 1) // 2) * ((W + 1) // 2), 18.0 * N * C * Cout * H * W)


def _aten_mode():
    from torch.utils._python_dispatch import TorchDispatchMode
    from torch.utils.flop_counter import flop_registry

    class AtenFlops(TorchDispatchMode):
        total = 0

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            kwargs = kwargs or {}
            out = func(*args, **kwargs)
            f = flop_registry.get(func._overloadpacket)
            if f is not None:
                self.total += f(*args, **kwargs, out_val=out)
            return out

    return AtenFlops()


@contextlib.contextmanager
def counting(aten=True):
    """Tally every native launch (and, with aten=True, every aten matmul / convolution,
    counted with torch.utils.flop_counter's formulas) issued inside the block."""
    t = Tally()
    _ACTIVE.append(t)
    mode = _aten_mode() if aten else contextlib.nullcontext()
    try:
        with mode:
            yield t
    finally:
        _ACTIVE.remove(t)
        if aten:
            t.aten = float(mode.total)
