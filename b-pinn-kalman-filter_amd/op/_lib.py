"""ctypes binding of the C ABI `libbpk.so` (declared in include/bpk.h).

The reference built its native ops with `torch.utils.cpp_extension.load` at
import time (op/upfirdn2d.py:10-17, op/fused_act.py:11-17, op/grid_sample.py:8-13,
op/ns_step.py:11-17).  Here the HIP library is prebuilt in-tree (see
`bpk_build.build()`), and this module binds it with ctypes: argument types are
generated from the prototypes in include/bpk.h, so the header stays the single
source of truth for the boundary.

There is no CPU fallback: every op requires HIP tensors, and a missing library
raises at first use.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

from . import _hipenv  # noqa: F401  (HIP runtime settings: before torch touches the device)
import torch  # noqa: E402

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_REPO_ROOT = os.path.dirname(_PKG_ROOT)
LIB_PATH = os.environ.get("BPK_LIB", os.path.join(_PKG_ROOT, "lib", "libbpk.so"))
HEADER_PATH = os.path.join(_REPO_ROOT, "include", "bpk.h")

_CTYPES = {
    "void": None,
    "int": ctypes.c_int,
    "int64_t": ctypes.c_int64,
    "uint64_t": ctypes.c_uint64,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "const char*": ctypes.c_char_p,
}

_PROTO_RE = re.compile(r"^\s*(const char\*|int64_t|int|void)\s+(bpk_\w+)\s*\(([^;]*?)\)\s*;", re.M | re.S)


def _ctype_of(decl: str):
    decl = " ".join(decl.split())
    if "*" in decl:
        return ctypes.c_void_p
    typ = decl.rsplit(" ", 1)[0] if " " in decl else decl
    typ = typ.replace("const ", "")
    if typ not in _CTYPES:
        raise TypeError(f"bpk.h: unsupported parameter type in '{decl}'")
    return _CTYPES[typ]


def parse_header(path: str = HEADER_PATH) -> dict:
    """Return {name: (restype, [argtypes])} for every prototype in bpk.h."""
    with open(path) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    protos = {}
    for ret, name, args in _PROTO_RE.findall(text):
        args = args.strip()
        argtypes = [] if args in ("", "void") else [_ctype_of(a) for a in args.split(",")]
        protos[name] = (_CTYPES[ret], argtypes)
    return protos


class _Lib:
    def __init__(self):
        self._lock = threading.Lock()
        self._dll = None
        self._protos = None

    def load(self):
        if self._dll is not None:
            return self._dll
        with self._lock:
            if self._dll is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(
                        f"bpk: HIP library not found at {LIB_PATH}; build it with "
                        "`python -c 'import __graft_entry__ as g; g.build()'` "
                        "(or `make -C b-pinn-kalman-filter_amd/csrc`)")
                # torch first: its bundled HIP runtime (same SONAME) must be the one
                # libbpk.so binds to, so streams/pointers are shared.
                dll = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
                protos = parse_header()
                for name, (res, args) in protos.items():
                    fn = getattr(dll, name)
                    fn.restype = res
                    fn.argtypes = args
                self._protos = protos
                self._dll = dll
        return self._dll

    def __getattr__(self, name):
        if not name.startswith("bpk_"):
            raise AttributeError(name)
        return getattr(self.load(), name)


lib = _Lib()


def check(rc: int, what: str = "bpk"):
    if rc != 0:
        msg = lib.bpk_last_error()
        msg = msg.decode() if isinstance(msg, bytes) else str(msg)
        raise RuntimeError(f"{what}: {msg} (status {rc})")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def require_hip(*tensors, what="bpk op"):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(f"{what}: expected a HIP (cuda) tensor, got device {t.device}")


def exported_symbols() -> list:
    return sorted(parse_header().keys())


_PRUNE = True


def mark_inputs(ctx, *args):
    """Record, in a custom Function's forward, which arguments are tensors: the engine keeps
    one next_functions edge per tensor argument only, so want_grad needs the mapping."""
    if ctx is not None:
        pos, k = [], 0
        for a in args:
            pos.append(k if isinstance(a, torch.Tensor) else None)
            k += isinstance(a, torch.Tensor)
        ctx._bpk_tpos = pos


def want_grad(ctx, i: int) -> bool:
    """ctx.needs_input_grad[i], and the autograd engine will use that gradient in the current
    backward pass: torch.autograd.grad(out, inputs=x) -- the PINN residual's derivative
    passes -- never runs the parameters' AccumulateGrad nodes, so the weight / bias gradients
    of a custom Function need not be computed there (ctx.needs_input_grad is fixed at forward
    time and would say yes).  Functions whose forward did not call mark_inputs: no pruning."""
    if not ctx.needs_input_grad[i]:
        return False
    pos = getattr(ctx, "_bpk_tpos", None)
    if not _PRUNE or pos is None or i >= len(pos) or pos[i] is None:
        return True
    nf = ctx.next_functions
    if pos[i] >= len(nf):
        return True
    node = nf[pos[i]][0]
    if node is None:
        return True
    try:
        return bool(torch._C._will_engine_execute_node(node))
    except RuntimeError:
        return True
