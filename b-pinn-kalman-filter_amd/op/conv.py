"""3x3 convolution on the fused Winograd F(2x2,3x3) MFMA kernel (csrc/conv_winograd.hip), or
on the small-channel VALU kernel (csrc/conv_small.hip) when Cin <= 4 or Cout <= 4.

`conv3x3(x, weight, bias=None)` == F.conv2d(x, weight, bias, stride=1, padding=1) for
fp32 NCHW HIP tensors whose shape the kernel supports (`supported(...)`).  Backward: the
input gradient is the same Winograd forward kernel on the flipped, transposed filter and
the weight gradient the Winograd split-K kernel (csrc/conv_winograd_wgrad.hip) when the
shapes qualify, else the implicit-GEMM kernels (csrc/conv_igemm.hip); MIOpen only for what no
native kernel takes (groups, dilation, non-fp32).  The filter
transform U = G w G^T is cached on the weight tensor itself (keyed by its version counter, which
every in-place update such as an optimizer step bumps), so a sampler that never changes
its weights transforms each filter once.
"""
from __future__ import annotations

import contextlib
import functools
import os

import torch
import torch.nn.functional as F
from torch.autograd.function import once_differentiable

from . import flops
from ._lib import check, lib, require_hip, stream_ptr, mark_inputs, want_grad


def _shape_ok(x, weight):
    return (x.dtype == torch.float32 and weight.dtype == torch.float32 and x.dim() == 4
            and tuple(weight.shape[2:]) == (3, 3) and x.is_cuda and weight.shape[1] == x.shape[1])


def wino_supported(x, weight):
    if not _shape_ok(x, weight):
        return False
    N, C, H, W = x.shape
    return bool(lib.bpk_conv3x3_wino_supported(N, C, weight.shape[0], H, W))


def wino_pair_supported(x, weight):
    """The 16-cin Winograd kernel's two-images-per-region form (8-pixel-wide images: CIFAR-10's
    8 x 8 level): one source, no GroupNorm statistics."""
    if not _shape_ok(x, weight):
        return False
    N, C, H, W = x.shape
    return bool(lib.bpk_conv3x3_wino_pair_supported(N, C, weight.shape[0], H, W))


def small_supported(x, weight):
    """The VALU small-channel kernel (csrc/conv_small.hip): Cin <= 4 or Cout <= 4."""
    if not _shape_ok(x, weight):
        return False
    N, C, H, W = x.shape
    return bool(lib.bpk_conv3x3_small_supported(N, C, weight.shape[0], H, W))


def supported(x, weight):
    """conv3x3() runs this conv natively: small-channel kernel or Winograd MFMA kernel."""
    return small_supported(x, weight) or wino_supported(x, weight)


_STATIC_FILTERS = None  # the registry of a capture in `static_filters` (else None)


@contextlib.contextmanager
def static_filters(registry: list):
    """Inside this block, a hipGraph capture reads the eagerly cached Winograd filter
    transforms instead of recording the transform kernels: each (weight, U) it uses is
    appended to `registry`, and the capturing code calls refresh_filters(registry) before
    replaying, which rewrites a U in place when its weight's version counter has moved (EMA
    copy_to, load_state_dict, an optimizer step).  The PC sampler's step graph uses this:
    its weights do not change between replays, so ~185 filter transforms per step go."""
    global _STATIC_FILTERS
    prev, _STATIC_FILTERS = _STATIC_FILTERS, registry
    try:
        yield registry
    finally:
        _STATIC_FILTERS = prev


def _transform_into(weight, U, ft):
    w = weight.detach().contiguous()
    Cout, Cin = (w.shape[1], w.shape[0]) if ft else (w.shape[0], w.shape[1])
    fn = lib.bpk_conv3x3_wino_filter_ft_f32 if ft else lib.bpk_conv3x3_wino_filter_f32
    check(fn(w.data_ptr(), U.data_ptr(), Cin, Cout, stream_ptr(w.device)), "conv3x3 filter")


def refresh_filters(registry: list):
    """Recompute, in place, the registered transforms whose weight changed since capture."""
    for i, (weight, U, ft, ver) in enumerate(registry):
        if weight._version != ver:
            _transform_into(weight, U, ft)
            registry[i] = (weight, U, ft, weight._version)


_FILTER_BATCH = None  # {(weight data_ptr, ft): (shape, U)} while a FilterBatch is active


class FilterBatch:
    """The Winograd filter transforms of every 3x3 / stride-1 / pad-1 conv weight of a module
    (forward and flipped), in static buffers refreshed by ONE launch
    (bpk_conv3x3_wino_filter_batch_f32) instead of one per conv call: a training step's
    weights change after every optimizer step, and the PINN step's graph recorded ~250
    transform launches.  `refresh()` transforms the current weights (capturable: the job
    table is device memory built once); inside `active()`, filter_transform returns these
    buffers -- the weights must not change in place within the block."""

    def __init__(self, module):
        jobs, self.map, self.params = [], {}, []
        dev = None
        for m in module.modules():
            if not (isinstance(m, torch.nn.Conv2d) and m.kernel_size == (3, 3)
                    and m.stride == (1, 1) and m.padding == (1, 1) and m.dilation == (1, 1)
                    and m.groups == 1):
                continue
            w = m.weight
            if not (w.is_cuda and w.dtype == torch.float32 and w.is_contiguous()):
                continue
            dev = w.device
            self.params.append(w)
            for ft in (False, True):
                Cout, Cin = (w.shape[1], w.shape[0]) if ft else (w.shape[0], w.shape[1])
                key = (w.data_ptr(), ft)
                if Cin % 8 or Cout % 16 or key in self.map:
                    continue  # not a Winograd filter shape
                CoutP = lib.bpk_conv3x3_wino_filter_bytes(Cin, Cout) // (16 * 4 * Cin)
                U = torch.empty((Cin, CoutP, 16), dtype=torch.float32, device=w.device)
                # keyed by storage (the conv paths pass detached views of the parameter)
                self.map[key] = (tuple(w.shape), U)
                jobs.append([w.data_ptr(), U.data_ptr(), Cin, Cout, CoutP, int(ft)])
        self.n = len(jobs)
        self.max_elems = max((j[2] * j[4] for j in jobs), default=0)
        self.jobs = torch.tensor(jobs, dtype=torch.int64).to(dev) if jobs else None
        self.ptrs = [w.data_ptr() for w in self.params]

    def valid_for(self, module) -> bool:
        """the recorded weights still live where the job table points (a weight replaced by
        another tensor is simply not found by filter_transform: per-call transforms)"""
        return all(w.data_ptr() == p for w, p in zip(self.params, self.ptrs))

    def refresh(self):
        if self.n:
            check(lib.bpk_conv3x3_wino_filter_batch_f32(
                self.jobs.data_ptr(), self.n, self.max_elems, stream_ptr(self.jobs.device)),
                "conv3x3 filter batch")

    @contextlib.contextmanager
    def active(self):
        global _FILTER_BATCH
        prev, _FILTER_BATCH = _FILTER_BATCH, self.map
        try:
            yield self
        finally:
            _FILTER_BATCH = prev


def filter_batch_for(module) -> "FilterBatch":
    """The FilterBatch of `module`, built on first use and kept on it (rebuilt when a weight
    tensor was replaced)."""
    fb = getattr(module, "_bpk_filter_batch", None)
    if fb is None or not fb.valid_for(module):
        fb = FilterBatch(module)
        object.__setattr__(module, "_bpk_filter_batch", fb)
    return fb


@contextlib.contextmanager
def batched_filters(module, enabled=True):
    """refresh() the module's FilterBatch and make it active for the block (a no-op when
    disabled or the module has no HIP 3x3 conv)."""
    if not enabled:
        yield None
        return
    fb = filter_batch_for(module)
    fb.refresh()
    with fb.active():
        yield fb


def filter_transform(weight, ft=False):
    """U [Cin, CoutP, 16] (CoutP = Cout rounded up to 64), cached on `weight` while its
    version counter is unchanged.  ft=True: the transform of _flip_t(weight) (the filter of
    the backward-data conv, Cin = weight.shape[0]), read from `weight` in place.  Inside an
    active FilterBatch: its static buffer."""
    fbm = _FILTER_BATCH
    if fbm is not None and weight.is_contiguous():
        e = fbm.get((weight.data_ptr(), bool(ft)))
        if e is not None and e[0] == tuple(weight.shape):
            return e[1]
    attr = "_bpk_wino_u_ft" if ft else "_bpk_wino_u"
    # under hipGraph capture the transform is recorded (and the cache left alone): replays
    # run after optimizer steps have rewritten the weight in place, so a cached U baked into
    # the graph would be stale from the second replay on -- unless the capture registers it
    # for refresh_filters (static_filters)
    capturing = torch.cuda.is_current_stream_capturing()
    cached = getattr(weight, attr, None)
    if capturing and _STATIC_FILTERS is not None and cached is not None \
            and cached[0] == weight._version:
        if not any(e[1] is cached[1] for e in _STATIC_FILTERS):
            _STATIC_FILTERS.append((weight, cached[1], ft, weight._version))
        return cached[1]
    if capturing:
        cached = None
    if cached is not None and cached[0] == weight._version:
        return cached[1]
    w = weight.detach().contiguous()
    Cout, Cin = (w.shape[1], w.shape[0]) if ft else (w.shape[0], w.shape[1])
    # Cout % 64 != 0: U is laid out for Cout rounded up to 64 (zero couts, never stored)
    CoutP = lib.bpk_conv3x3_wino_filter_bytes(Cin, Cout) // (16 * 4 * Cin)
    U = torch.empty((Cin, CoutP, 16), dtype=torch.float32, device=w.device)
    fn = lib.bpk_conv3x3_wino_filter_ft_f32 if ft else lib.bpk_conv3x3_wino_filter_f32
    check(fn(w.data_ptr(), U.data_ptr(), Cin, Cout, stream_ptr(w.device)), "conv3x3 filter")
    if not capturing:
        setattr(weight, attr, (weight._version, U))
    return U


GN_PART_COUNT = 128  # pixels per partial-statistics region (8 x 16)


def gn_partials(t):
    """(part [N, C, R, 2], R, count) attached to `t` by a stats-producing conv, or None if
    absent or stale (t modified in place since)."""
    p = getattr(t, "_bpk_gn_part", None)
    if p is None or p[3] != t._version:
        return None
    return p[:3]


def attach_gn_partials(t, part, R, cnt=GN_PART_COUNT):
    t._bpk_gn_part = (part, R, cnt, t._version)
    return t


def ensure_gn_partials(t):
    """gn_partials(t), computing them with one read of t (bpk_group_norm_chunk_partials_f32)
    when its producer attached none; None when the shape has no partials form."""
    p = gn_partials(t)
    if p is not None:
        return p
    if (t.dim() != 4 or not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous()
            or (t.shape[2] * t.shape[3]) % GN_PART_COUNT != 0):
        return None
    N, C, H, W = t.shape
    R = H * W // GN_PART_COUNT
    part = torch.empty((N, C, R, 2), dtype=torch.float32, device=t.device)
    check(lib.bpk_group_norm_chunk_partials_f32(t.data_ptr(), part.data_ptr(), N, C, H * W,
                                                stream_ptr(t.device)), "gn_partials")
    attach_gn_partials(t, part, R)
    return part, R, GN_PART_COUNT


def conv3x3_fwd_raw(x, weight, bias=None, skip=None, div=1.0, pre=None, stats=False, x2=None,
                    ft=False):
    """conv(a, weight) + bias, or with `skip`: (skip + (conv + bias)) / div (one launch),
    where a = x, or silu(x * s + t) with pre[n, c] = (s, t) (GroupNorm+SiLU fused in).
    stats=True also writes the GroupNorm partial statistics of the output (attached to it,
    see gn_partials) so the next GroupNorm skips its statistics pass.  ft=True: the filter
    is _flip_t(weight) (backward-data), without materialising it."""
    x = x.contiguous()
    N, C1, H, W = x.shape
    C = C1 if x2 is None else C1 + x2.shape[1]
    if x2 is not None:
        x2 = x2.contiguous()
        if x2.shape[0] != N or tuple(x2.shape[2:]) != (H, W) or C1 % 8:
            raise RuntimeError(f"conv3x3: second source {tuple(x2.shape)} vs {tuple(x.shape)}")
    Cout = weight.shape[1] if ft else weight.shape[0]
    U = filter_transform(weight, ft)
    y = torch.empty((N, Cout, H, W), dtype=x.dtype, device=x.device)
    b = None if bias is None else bias.detach().contiguous()
    sk = None if skip is None else skip.detach().contiguous()
    if sk is not None and sk.shape != y.shape:
        raise RuntimeError(f"conv3x3: skip {tuple(sk.shape)} != output {tuple(y.shape)}")
    pr = None if pre is None else pre.contiguous()
    if pr is not None and tuple(pr.shape) != (N, C, 2):
        raise RuntimeError(f"conv3x3: pre must be [N, Cin, 2], got {tuple(pr.shape)}")
    part = None
    if stats:
        R = (H // 8) * (W // 16)
        part = torch.empty((N, Cout, R, 2), dtype=torch.float32, device=x.device)
    # split-K over the input channels when the launch would leave most CUs idle (small
    # per-GPU batches at the 32^2 / 16^2 levels); the workspace comes from the caching
    # allocator (the graph's pool under capture)
    nws = lib.bpk_conv3x3_wino_splitk_bytes(N, C, C1 if x2 is not None else C, Cout, H, W)
    ws = torch.empty(nws // 4, dtype=torch.float32, device=x.device) if nws > 0 else None
    check(lib.bpk_conv3x3_wino_splitk_f32(
        x.data_ptr(), None if x2 is None else x2.data_ptr(), C1,
        None if pr is None else pr.data_ptr(), U.data_ptr(),
        None if b is None else b.data_ptr(), None if sk is None else sk.data_ptr(), float(div),
        y.data_ptr(), None if part is None else part.data_ptr(),
        None if ws is None else ws.data_ptr(), N, C, Cout, H, W,
        stream_ptr(x.device)), "conv3x3_wino")
    flops.wino3x3("wino_dgrad" if ft else "wino_fwd", N, C, Cout, H, W)
    if part is not None:
        attach_gn_partials(y, part, R)
    return y


_WGRAD = True  # 3x3 weight gradients on the Winograd kernel (False: MIOpen / igemm)


def wgrad_supported(x, weight):
    """weight: the weight tensor or just its shape"""
    if not _WGRAD:
        return False
    if x.dtype != torch.float32 or x.dim() != 4 or not x.is_cuda:
        return False
    N, C, H, W = x.shape
    cout = weight[0] if isinstance(weight, (tuple, list, torch.Size)) else weight.shape[0]
    return bool(lib.bpk_conv3x3_wino_wgrad_supported(N, C, cout, H, W))


def conv3x3_wgrad_raw(x, gy, wshape, bias_grad=False, pre=None):
    """dw [Cout, Cin, 3, 3] of conv3x3(x, w) for the output gradient gy (Winograd split-K,
    csrc/conv_winograd_wgrad.hip); == torch.nn.grad.conv2d_weight(x, wshape, gy, padding=1).
    bias_grad=True: returns (dw, db) with db = gy.sum((0, 2, 3)) from the same kernel.
    pre [N, Cin, 2] = (s, t): the convolved input is silu(x * s + t) (the GroupNorm+SiLU
    prologue of gn_silu_conv3x3_ad), applied in the kernel's patch load."""
    x = x.detach().contiguous()
    gy = gy.detach().contiguous()
    N, C, H, W = x.shape
    Cout = wshape[0]
    if tuple(gy.shape) != (N, Cout, H, W) or tuple(wshape[1:]) != (C, 3, 3):
        raise RuntimeError(f"conv3x3_wgrad: x {tuple(x.shape)}, gy {tuple(gy.shape)}, "
                           f"w {tuple(wshape)}")
    nbytes = lib.bpk_conv3x3_wino_wgrad_workspace_bytes(N, C, Cout, H, W)
    ws = torch.empty(nbytes // 4, dtype=torch.float32, device=x.device)
    dw = torch.empty((Cout, C, 3, 3), dtype=torch.float32, device=x.device)
    db = torch.empty((Cout,), dtype=torch.float32, device=x.device) if bias_grad else None
    pr = None if pre is None else pre.detach().contiguous()
    if pr is not None and tuple(pr.shape) != (N, C, 2):
        raise RuntimeError(f"conv3x3_wgrad: pre must be [N, Cin, 2], got {tuple(pr.shape)}")
    check(lib.bpk_conv3x3_wino_wgrad_pre_f32(
        x.data_ptr(), None if pr is None else pr.data_ptr(), gy.data_ptr(), dw.data_ptr(),
        None if db is None else db.data_ptr(), ws.data_ptr(), N, C, Cout, H, W,
        stream_ptr(x.device)), "conv3x3_wgrad")
    flops.wino3x3("wino_wgrad", N, C, Cout, H, W)
    return (dw, db) if bias_grad else dw


def conv3x3_small_raw(x, weight, bias=None, pre=None):
    """conv(a, weight) + bias on the small-channel kernel, a = x or silu(x * s + t)."""
    x = x.contiguous()
    N, C, H, W = x.shape
    Cout = weight.shape[0]
    w = weight.detach().contiguous()
    y = torch.empty((N, Cout, H, W), dtype=x.dtype, device=x.device)
    b = None if bias is None else bias.detach().contiguous()
    pr = None if pre is None else pre.contiguous()
    if pr is not None and tuple(pr.shape) != (N, C, 2):
        raise RuntimeError(f"conv3x3: pre must be [N, Cin, 2], got {tuple(pr.shape)}")
    check(lib.bpk_conv3x3_small_f32(
        x.data_ptr(), None if pr is None else pr.data_ptr(), w.data_ptr(),
        None if b is None else b.data_ptr(), y.data_ptr(), N, C, Cout, H, W,
        stream_ptr(x.device)), "conv3x3_small")
    flops.add("valu_conv3x3", 18.0 * N * C * Cout * H * W)
    return y


# ------------------------------------------------ general convolutions on the MFMA (igemm)
_IGEMM = True  # the implicit-GEMM kernels for the shapes below (False: MIOpen only)


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(int(e) for e in v)


def igemm_supported(x, w, stride=1, padding=0, dilation=1, groups=1):
    """The implicit-GEMM MFMA kernels (csrc/conv_igemm.hip) run conv2d(x, w) and all of its
    derivatives: fp32 NCHW HIP tensors, groups = 1, dilation = 1, zero padding.  `w`: the
    weight tensor or its shape."""
    wshape = tuple(w) if isinstance(w, (tuple, list, torch.Size)) else tuple(w.shape)
    if isinstance(w, torch.Tensor) and w.dtype != torch.float32:
        return False
    if not (_IGEMM and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
            and len(wshape) == 4 and int(groups) == 1
            and _pair(dilation) == (1, 1) and wshape[1] == x.shape[1]
            and x.shape[2] + 2 * _pair(padding)[0] >= wshape[2]
            and x.shape[3] + 2 * _pair(padding)[1] >= wshape[3]):
        return False
    return _igemm_shape_ok(tuple(x.shape), tuple(int(v) for v in wshape), _pair(stride),
                           _pair(padding))


@functools.lru_cache(maxsize=4096)
def _igemm_shape_ok(xshape, wshape, s, p):
    """The kernels' own limits (32-bit index ranges, tile counts): the workspace query of the
    forward, its adjoint and the weight gradient answers -1 for a shape they cannot run, and
    such a conv stays on MIOpen instead of raising."""
    N, C, H, W = xshape
    Co, _, KH, KW = wshape
    Ho, Wo = (H + 2 * p[0] - KH) // s[0] + 1, (W + 2 * p[1] - KW) // s[1] + 1
    return all(lib.bpk_conv2d_igemm_workspace_bytes(m, N, C, H, W, Co, KH, KW, s[0], s[1], p[0],
                                                    p[1], Ho, Wo, 1) >= 0 for m in (0, 1, 2))


def _igemm_ws(mode, N, C, H, W, Co, KH, KW, s, p, Ho, Wo, bias_grad, device):
    nbytes = lib.bpk_conv2d_igemm_workspace_bytes(mode, N, C, H, W, Co, KH, KW, s[0], s[1],
                                                  p[0], p[1], Ho, Wo, int(bias_grad))
    if nbytes < 0:
        raise RuntimeError(f"conv2d_igemm: unsupported shape x [{N}, {C}, {H}, {W}], "
                           f"w [{Co}, {C}, {KH}, {KW}]")
    return torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=device)


def conv2d_igemm_raw(x, w, bias=None, stride=1, padding=0):
    """F.conv2d(x, w, bias, stride, padding) on the implicit-GEMM MFMA kernel (no autograd)."""
    s, p = _pair(stride), _pair(padding)
    x = x.detach().contiguous()
    w = w.detach().contiguous()
    N, C, H, W = x.shape
    Co, _, KH, KW = w.shape
    Ho, Wo = (H + 2 * p[0] - KH) // s[0] + 1, (W + 2 * p[1] - KW) // s[1] + 1
    b = None if bias is None else bias.detach().contiguous()
    y = torch.empty((N, Co, Ho, Wo), dtype=torch.float32, device=x.device)
    ws = _igemm_ws(0, N, C, H, W, Co, KH, KW, s, p, Ho, Wo, False, x.device)
    check(lib.bpk_conv2d_igemm_fwd_f32(x.data_ptr(), w.data_ptr(),
                                       None if b is None else b.data_ptr(), y.data_ptr(),
                                       ws.data_ptr(), N, C, H, W, Co, KH, KW, s[0], s[1], p[0],
                                       p[1], Ho, Wo, stream_ptr(x.device)), "conv2d_igemm_fwd")
    flops.add("igemm_fwd", 2.0 * N * Co * C * KH * KW * Ho * Wo)
    return y


def conv2d_input_igemm_raw(xshape, w, gy, stride=1, padding=0):
    """torch.nn.grad.conv2d_input(xshape, w, gy, stride, padding) -- the conv's adjoint, i.e.
    F.conv_transpose2d(gy, w) cropped / extended to xshape -- on the MFMA kernel."""
    s, p = _pair(stride), _pair(padding)
    w = w.detach().contiguous()
    gy = gy.detach().contiguous()
    N, C, H, W = (int(v) for v in xshape)
    Co, _, KH, KW = w.shape
    Ho, Wo = gy.shape[2], gy.shape[3]
    gx = torch.empty((N, C, H, W), dtype=torch.float32, device=gy.device)
    ws = _igemm_ws(1, N, C, H, W, Co, KH, KW, s, p, Ho, Wo, False, gy.device)
    check(lib.bpk_conv2d_igemm_dgrad_f32(gy.data_ptr(), w.data_ptr(), gx.data_ptr(),
                                         ws.data_ptr(), N, C, H, W, Co, KH, KW, s[0], s[1],
                                         p[0], p[1], Ho, Wo, stream_ptr(gy.device)),
          "conv2d_igemm_dgrad")
    flops.add("igemm_dgrad", 2.0 * N * Co * C * KH * KW * Ho * Wo)
    return gx


def conv2d_weight_igemm_raw(x, wshape, gy, stride=1, padding=0, bias_grad=False):
    """(torch.nn.grad.conv2d_weight(x, wshape, gy, stride, padding), gy.sum((0, 2, 3)) or
    None) from one MFMA kernel (the bias gradient is an extra GEMM column of ones)."""
    s, p = _pair(stride), _pair(padding)
    x = x.detach().contiguous()
    gy = gy.detach().contiguous()
    N, C, H, W = x.shape
    Co, _, KH, KW = (int(v) for v in wshape)
    Ho, Wo = gy.shape[2], gy.shape[3]
    dw = torch.empty((Co, C, KH, KW), dtype=torch.float32, device=x.device)
    db = torch.empty((Co,), dtype=torch.float32, device=x.device) if bias_grad else None
    ws = _igemm_ws(2, N, C, H, W, Co, KH, KW, s, p, Ho, Wo, bias_grad, x.device)
    check(lib.bpk_conv2d_igemm_wgrad_f32(x.data_ptr(), gy.data_ptr(), dw.data_ptr(),
                                         None if db is None else db.data_ptr(), ws.data_ptr(),
                                         N, C, H, W, Co, KH, KW, s[0], s[1], p[0], p[1], Ho, Wo,
                                         stream_ptr(x.device)), "conv2d_igemm_wgrad")
    flops.add("igemm_wgrad", 2.0 * N * Co * C * KH * KW * Ho * Wo)
    return dw, db


def _small_cout_wgrad_ok(x, wshape, s, p):
    Co, C, KH, KW = wshape
    return (Co <= 4 and KH == KW and KH in (1, 3) and s == (1, 1) and p == (KH // 2, KW // 2)
            and bool(lib.bpk_conv2d_wgrad_small_cout_supported(x.shape[0], C, Co, x.shape[2],
                                                                x.shape[3], KH)))


def conv2d_weight_small_cout_raw(x, wshape, gy, bias_grad=False):
    """(dw, db or None) of a K x K / stride 1 / pad K // 2 conv into Cout <= 4 channels on the
    streaming VALU kernel (csrc/conv_small.hip)."""
    x = x.detach().contiguous()
    gy = gy.detach().contiguous()
    N, C, H, W = x.shape
    Co, _, K, _ = (int(v) for v in wshape)
    dw = torch.empty((Co, C, K, K), dtype=torch.float32, device=x.device)
    db = torch.empty((Co,), dtype=torch.float32, device=x.device) if bias_grad else None
    nb = lib.bpk_conv2d_wgrad_small_cout_workspace_bytes(N, C, Co, K)
    ws = torch.empty(max(nb // 4, 1), dtype=torch.float32, device=x.device)
    check(lib.bpk_conv2d_wgrad_small_cout_f32(x.data_ptr(), gy.data_ptr(), dw.data_ptr(),
                                              None if db is None else db.data_ptr(),
                                              ws.data_ptr(), N, C, Co, H, W, K,
                                              stream_ptr(x.device)), "conv2d_wgrad_small_cout")
    flops.add("valu_wgrad", 2.0 * N * Co * C * K * K * H * W)
    return dw, db


# Kernel selection per distinct call.  Among native kernels (Winograd vs implicit GEMM on small
# images) the first eager call of each (op, shapes) times the candidates once and caches the
# faster; under graph capture an unseen call takes the first candidate.  MIOpen is not a
# candidate (round 4): every conv the networks run has a native kernel, and timing MIOpen's
# candidates cost seconds per process (immediate mode falls back to its naive kernels for
# several backward shapes: 0.2 s per call) for, at best, 0.3 % of a sampler step (the two
# stride-2 FIR-down shapes at B = 64, profiles/r04_stride2_igemm_vs_miopen.txt).
# `library_candidates()` puts MIOpen back in the igemm-vs-library choices (A/B tools).
_CHOICE: dict = {}        # agreed choices (broadcast from rank 0 under torch.distributed)
_CHOICE_LOCAL: dict = {}  # choices made inside local_choices(): this rank's own, never agreed


def _time_us(fn, reps=3):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


# Small images (H * W <= 32 x 32, the PINN pyramids' lower levels, CIFAR's 8^2 / 4^2): the
# Winograd kernels' per-workgroup set-up is a large share of a short launch, so 3x3 convs
# there are timed against the implicit-GEMM kernel once per distinct call and the faster
# kept.
_SEL3 = True
_SEL3_MAX_HW = 32 * 32


def _small_img(x):
    return _SEL3 and _IGEMM and x.shape[2] * x.shape[3] <= _SEL3_MAX_HW


# Reproducibility of the per-call choice (the timing is noisy, so two runs -- or two ranks --
# could take different kernels for the same call and differ in the last bits):
#  * BPK_CONV_PICK=first: no timing, always the first candidate (igemm / Winograd);
#  * BPK_CONV_TABLE=path.json: choices are read from the file at import and every new
#    choice is written back (a run can replay another run's table exactly);
#  * under torch.distributed with world size > 1 the choice of rank 0 is broadcast, so
#    every rank runs the same kernels (the calls are SPMD: every rank reaches each new key
#    in the same order; code only some ranks run goes inside `local_choices()`).
_PICK_FIRST = os.environ.get("BPK_CONV_PICK", "") == "first"
_TABLE_PATH = os.environ.get("BPK_CONV_TABLE")


def _key_str(key):
    return repr(key)


def _load_table():
    if not _TABLE_PATH or not os.path.exists(_TABLE_PATH):
        return {}
    import json
    with open(_TABLE_PATH) as f:
        return {k: int(v) for k, v in json.load(f).items()}


_TABLE = _load_table()


def _save_table():
    import json
    tmp = _TABLE_PATH + ".tmp"
    with open(tmp, "w") as f:
        json.dump(_TABLE, f, indent=0, sort_keys=True)
    os.replace(tmp, _TABLE_PATH)


_LOCAL_ONLY = [False]
_NATIVE_ONLY = [True]


@contextlib.contextmanager
def native_only():
    """Inside this block the igemm-vs-MIOpen choices take the implicit-GEMM kernel (the choices
    among native kernels stay timed) even inside `library_candidates()`: a step captured in a
    hipGraph (the PINN step, losses.get_pinn_step_fn(graph=True)) holds only libbpk / aten
    kernels and no MIOpen workspace or find-db state."""
    prev, _NATIVE_ONLY[0] = _NATIVE_ONLY[0], True
    try:
        yield
    finally:
        _NATIVE_ONLY[0] = prev


@contextlib.contextmanager
def library_candidates():
    """Inside this block MIOpen is timed against the implicit-GEMM kernel again (per call, the
    faster kept): for A/B measurements only, the product default is native kernels."""
    prev, _NATIVE_ONLY[0] = _NATIVE_ONLY[0], False
    try:
        yield
    finally:
        _NATIVE_ONLY[0] = prev


@contextlib.contextmanager
def local_choices():
    """Inside this block new choices are NOT broadcast: for code that only some ranks run
    (a rank-0-only measurement), where a collective would wait for ranks that never come."""
    prev, _LOCAL_ONLY[0] = _LOCAL_ONLY[0], True
    try:
        yield
    finally:
        _LOCAL_ONLY[0] = prev


def _rank() -> int:
    import torch.distributed as dist
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def _agree(c: int) -> int:
    """Rank 0's choice on every rank (identity when not distributed)."""
    import torch.distributed as dist
    if (_LOCAL_ONLY[0] or not (dist.is_available() and dist.is_initialized())
            or dist.get_world_size() == 1):
        return c
    dev = "cpu" if dist.get_backend() == "gloo" else torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([c], dtype=torch.int64, device=dev)
    dist.broadcast(t, 0)
    return int(t.item())


def _decide(key, timers):
    """Index of the candidate to run for `key`: cached, from the table, or timed once
    (None under graph capture for a key never decided eagerly).  A choice made inside
    `local_choices()` is kept apart from the agreed ones, so a later SPMD call of the same key
    still goes through the broadcast on every rank (otherwise rank 0 would skip it and the
    other ranks would wait in it)."""
    local = _LOCAL_ONLY[0]
    c = _CHOICE.get(key)
    if c is None and local:
        c = _CHOICE_LOCAL.get(key)
    if c is not None:
        return c
    ks = _key_str(key)
    if ks in _TABLE and 0 <= _TABLE[ks] < len(timers):
        c = _TABLE[ks]
    elif _PICK_FIRST:
        c = 0
    elif torch.cuda.is_current_stream_capturing():
        return None
    else:
        with torch.no_grad():
            ts = [_time_us(f) for f in timers]
        c = _agree(min(range(len(timers)), key=ts.__getitem__))
        if _TABLE_PATH and not local:  # a table entry written by another candidate list
            _TABLE[ks] = c             # (out of range above) is overwritten here
            if _rank() == 0:  # one writer (every rank holds the same, agreed choices)
                _save_table()
    (_CHOICE_LOCAL if local else _CHOICE)[key] = c
    return c


def _pick_any(key, cands):
    """cands[i]() for the candidate the cached per-key timing says is fastest (the first
    one under graph capture for a key never timed eagerly)."""
    c = _decide(key, cands)
    return cands[0 if c is None else c]()


def _pick(key, run_ig, run_mi):
    """run_ig() or run_mi(), whichever the cached per-key timing says is faster (ties: igemm)."""
    if _NATIVE_ONLY[0]:
        return run_ig()
    c = _decide(key, [run_ig, run_mi])
    return run_mi() if c == 1 else run_ig()


def conv2d_select(x, w, bias, stride, padding):
    """F.conv2d(x, w, bias, stride, padding) (no autograd) on the faster of igemm / MIOpen."""
    s, p = _pair(stride), _pair(padding)
    key = ("fwd", tuple(x.shape), tuple(w.shape), s, p, bias is not None)
    b = None if bias is None else bias.detach()
    return _pick(key, lambda: conv2d_igemm_raw(x, w, b, s, p),
                 lambda: F.conv2d(x.detach(), w.detach(), b, s, p))


def conv2d_input_select(xshape, w, gy, stride, padding):
    s, p = _pair(stride), _pair(padding)
    xshape = tuple(int(v) for v in xshape)
    key = ("dgrad", xshape, tuple(w.shape), s, p)

    def ig():
        return conv2d_input_igemm_raw(xshape, w, gy, s, p)
    N, C, H, W = xshape
    if (C <= 4 and tuple(w.shape[2:]) == (3, 3) and s == (1, 1) and p == (1, 1)
            and bool(lib.bpk_conv3x3_small_supported(N, w.shape[0], C, H, W))):
        # into <= 4 channels: the conv of gy with the flipped, transposed filter on the
        # small-Cout streaming kernel (the PINN heads' input gradients), timed against igemm
        ig_any = ig
        ig = lambda: _pick_any(("dsc",) + key[1:], [  # noqa: E731
            lambda: conv3x3_small_raw(gy.detach().contiguous(), _flip_t(w.detach()).contiguous()),
            ig_any])
    return _pick(key, ig,
                 lambda: torch.nn.grad.conv2d_input(xshape, w.detach(), gy.detach(), s, p))


def conv2d_weight_select(x, wshape, gy, stride, padding, bias_grad):
    s, p = _pair(stride), _pair(padding)
    wshape = tuple(int(v) for v in wshape)
    key = ("wgrad", tuple(x.shape), wshape, s, p, bool(bias_grad))

    def mi():
        dw = torch.nn.grad.conv2d_weight(x.detach(), wshape, gy.detach(), s, p)
        return dw, (gy.detach().sum((0, 2, 3)) if bias_grad else None)

    def ig():
        return conv2d_weight_igemm_raw(x, wshape, gy, s, p, bias_grad)
    if _small_cout_wgrad_ok(x, wshape, s, p):  # few output channels: streaming kernel vs igemm
        ig_any = ig
        ig = lambda: _pick_any(("wsc",) + key[1:], [  # noqa: E731
            lambda: conv2d_weight_small_cout_raw(x, wshape, gy, bias_grad), ig_any])
    return _pick(key, ig, mi)


def _flip_t(w):
    """[Cout, Cin, 3, 3] -> the flipped, transposed filter [Cin, Cout, 3, 3]: backward-data of
    a 3x3 / stride-1 / pad-1 conv is the forward conv of the output gradient with it."""
    return w.flip(2, 3).transpose(0, 1)


def _fwd_impl(x, w, bias=None, skip=None, div=1.0):
    """conv(x, w) + bias [-> (skip + .) / div] without autograd: Winograd MFMA kernel,
    small-channel kernel, or MIOpen for the other shapes."""
    w = w.detach().contiguous()
    if wino_supported(x, w) or wino_pair_supported(x, w):
        if _small_img(x) and igemm_supported(x, w, 1, 1):
            def ig():
                y = conv2d_igemm_raw(x, w, None if bias is None else bias.detach(), 1, 1)
                if skip is not None:
                    from .norm_act import residual_rescale
                    y = residual_rescale(skip.detach(), y, None, div)
                return y
            key = ("f3", tuple(x.shape), tuple(w.shape), bias is not None, skip is not None)
            return _pick_any(key, [lambda: conv3x3_fwd_raw(x.detach(), w, bias, skip, div), ig])
        return conv3x3_fwd_raw(x.detach(), w, bias, skip, div)
    with torch.no_grad():
        if small_supported(x, w):
            y = conv3x3_small_raw(x.detach(), w, bias)
        elif igemm_supported(x, w, 1, 1):
            y = conv2d_select(x, w, bias, 1, 1)
        else:
            y = F.conv2d(x.detach(), w, None if bias is None else bias.detach(), padding=1)
        if skip is not None:
            from .norm_act import residual_rescale
            y = residual_rescale(skip.detach(), y, None, div)
    return y


def _wgrad_impl(x, gy, wshape, want_b):
    """(dw, db or None) without autograd: the Winograd weight gradient (+ bias) when the
    shape qualifies, MIOpen backward-weights otherwise."""
    if wgrad_supported(x, tuple(wshape)):
        # small images, and couts past a 64-cout block (the Winograd kernel's idle waves),
        # are timed against the implicit GEMM once per distinct call
        if ((_small_img(x) or wshape[0] % 64) and x.is_cuda and x.dtype == torch.float32
                and igemm_supported(x, tuple(wshape), 1, 1)):
            key = ("w3", tuple(x.shape), tuple(wshape))
            dw, db = _pick_any(key, [
                lambda: conv3x3_wgrad_raw(x, gy, wshape, bias_grad=True),
                lambda: conv2d_weight_igemm_raw(x, tuple(wshape), gy, 1, 1, True)])
            return dw, (db if want_b else None)
        dw, db = conv3x3_wgrad_raw(x, gy, wshape, bias_grad=True)
        return dw, (db if want_b else None)
    elif igemm_supported(x, tuple(wshape), 1, 1):
        return conv2d_weight_select(x, tuple(wshape), gy, 1, 1, want_b)
    else:
        with torch.no_grad():
            dw = torch.nn.grad.conv2d_weight(x.detach(), wshape, gy.detach(), padding=1)
    return dw, (gy.detach().sum((0, 2, 3)) if want_b else None)


def _fwd_ft_impl(x, w):
    """conv3x3(x, _flip_t(w)) without autograd; the Winograd filter transform reads w
    flipped and transposed in place when the shape qualifies."""
    w = w.detach()
    N, C, H, W = x.shape
    if (C == w.shape[0] and x.is_cuda and x.dtype == torch.float32
            and (bool(lib.bpk_conv3x3_wino_supported(N, C, w.shape[1], H, W))
                 or bool(lib.bpk_conv3x3_wino_pair_supported(N, C, w.shape[1], H, W)))):
        if (_small_img(x) and _IGEMM and w.dtype == torch.float32
                and _igemm_shape_ok((N, w.shape[1], H, W), tuple(w.shape), (1, 1), (1, 1))):
            key = ("d3", tuple(x.shape), tuple(w.shape))
            return _pick_any(key, [lambda: conv3x3_fwd_raw(x.detach(), w, ft=True),
                                   lambda: conv2d_input_igemm_raw((N, w.shape[1], H, W), w, x, 1, 1)])
        return conv3x3_fwd_raw(x.detach(), w, ft=True)
    if (_IGEMM and x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32
            and _igemm_shape_ok((N, w.shape[1], H, W), tuple(w.shape), (1, 1), (1, 1))):
        # conv3x3(x, flip_t(w)) is the adjoint of conv3x3(., w): the dgrad kernel, no flip
        return conv2d_input_select((N, w.shape[1], H, W), w, x, 1, 1)
    return _fwd_impl(x, _flip_t(w))


_FT = True  # the filter transform reads the weight flipped / transposed (False: a copy)


def _conv_ft_any(x, w):
    """conv3x3(x, _flip_t(w)) -- the backward-data conv -- recorded for autograd when grad
    mode is on, else the raw kernels."""
    if not _FT:
        return _conv_any(x, _flip_t(w))
    if torch.is_grad_enabled():
        return _Conv3x3FT.apply(x, w)
    return _fwd_ft_impl(x, w)


class _Conv3x3FT(torch.autograd.Function):
    """y = conv3x3(x, _flip_t(w)) for w [Co, Ci, 3, 3] (x has Co channels).  Adjoint:
    d/dx = conv3x3(gy, w) (flip_t is an involution); d/dw = _flip_t(wgrad(x, gy)), which is
    the weight gradient with the roles of input and output gradient exchanged,
    d/dw[a][b][r][s] = sum_q x[a](q) gy[b](q + (r - 1, s - 1)) = wgrad(gy, x) -- computed in
    w's own layout (no flip launch, and a contiguous gradient AccumulateGrad can take without
    a copy).  Both differentiable again (second derivatives of the PINN residual)."""

    @staticmethod
    def forward(ctx, x, w):
        mark_inputs(ctx, x, w)
        ctx.save_for_backward(x, w)
        return _fwd_ft_impl(x, w)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = gw = None
        if want_grad(ctx, 0):
            gx = _conv_any(gy, w)
        if want_grad(ctx, 1):
            if torch.is_grad_enabled():
                gw = _Wgrad3x3.apply(gy, x, tuple(w.shape))
            elif not _defer_wgrad(w, gy, x, ("3x3",)):
                gw = _wgrad_impl(gy, x, tuple(w.shape), False)[0]
        return gx, gw


def _conv_any(x, w):
    """conv3x3(x, w) recorded for autograd when grad mode is on (higher derivatives), else
    the raw kernels."""
    if torch.is_grad_enabled():
        return _Conv3x3.apply(x, w.contiguous(), None, None, 1.0)
    return _fwd_impl(x, w)


class _Conv3x3(torch.autograd.Function):
    """y = (skip + conv3x3(x, w) + bias) / div (skip optional).  Its backward is written in
    terms of this op and _Wgrad3x3, both differentiable again, so second and higher
    derivatives (the PINN residual, create_graph=True) stay on 3x3 convs and weight
    gradients -- never on the batch/channel-swapped 'convolutions' with H x W kernels that
    a generic double backward of a convolution produces."""

    @staticmethod
    def forward(ctx, x, weight, bias, skip, div):
        mark_inputs(ctx, x, weight, bias, skip, div)
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.bias_leaf = bias if bias is not None and bias.is_leaf else None
        ctx.div = float(div)
        return _fwd_impl(x, weight, bias, skip, div)

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gx = gw = gb = gs = None
        if ctx.div != 1.0:
            gy = gy / ctx.div
        if want_grad(ctx, 3):
            gs = gy
        want_b = ctx.has_bias and want_grad(ctx, 2)
        if want_grad(ctx, 0):
            gx = _conv_ft_any(gy, weight)
        if torch.is_grad_enabled():
            if want_grad(ctx, 1):
                gw = _Wgrad3x3.apply(x, gy, tuple(weight.shape))
            if want_b:
                gb = gy.sum((0, 2, 3))
        elif (want_grad(ctx, 1) and (not want_b or ctx.bias_leaf is not None)
              and _defer_wgrad(weight, x, gy, ("3x3",), ctx.bias_leaf if want_b else None)):
            pass  # weight (and bias) gradients deferred to the end of the backward pass
        elif want_grad(ctx, 1) or want_b:
            dw, gb = _wgrad_impl(x, gy, tuple(weight.shape), want_b)
            gw = dw if want_grad(ctx, 1) else None
        return gx, gw, gb, gs, None


class _Wgrad3x3(torch.autograd.Function):
    """dw = sum over (n, p) of gy[n, co, p] x[n, ci, p + (r, s)] (the weight gradient of the
    3x3 / pad-1 conv).  Linear in x and in gy: for an incoming ggw,
    d/dx = conv3x3(gy, flip_t(ggw)) and d/dgy = conv3x3(x, ggw)."""

    @staticmethod
    def forward(ctx, x, gy, wshape):
        mark_inputs(ctx, x, gy, wshape)
        ctx.save_for_backward(x, gy)
        return _wgrad_impl(x, gy, wshape, False)[0]

    @staticmethod
    def backward(ctx, ggw):
        x, gy = ctx.saved_tensors
        gx = ggy = None
        if want_grad(ctx, 0):
            gx = _conv_ft_any(gy, ggw)
        if want_grad(ctx, 1):
            ggy = _conv_any(x, ggw)
        return gx, ggy, None


# ---------------------------------------------------------------- deferred weight gradients
# The PINN step's final backward (losses.get_pinn_step_fn) reaches almost every conv weight
# twice: through the conv of the forward and through its backward-data conv recorded by the
# residual's first-order pass (create_graph).  Each contribution is a weight-gradient launch
# (plus, at small batches, its split-K reduce), and autograd adds the two in the weight's input
# buffer -- three to five launches per weight, ~130 weights.  Inside
# `deferred_weight_grads()` the backward nodes only record the (input, output-gradient) pair of
# a leaf weight (and of its bias); when the block ends, each weight's pairs run as ONE
# weight-gradient launch over both sources (bpk_conv3x3_wino_wgrad2_f32 /
# bpk_conv2d_igemm_wgrad2_f32: the K sum runs over the images of both pairs) and the result is
# written to .grad (added when .grad already holds a gradient).  Per distinct shape the
# two-source launch is timed once against the two separate launches + add, and the faster kept.
# Same sums as autograd's up to the order of the additions (one K sum instead of two plus an
# add); the bias gradient comes from the forward conv's pair alone, as before.
_DEFER = [None]


class _Deferral:
    def __init__(self):
        self.entries = {}  # id(weight) -> [weight, bias leaf or None, kind, [(X, GY, has_b)]]


@contextlib.contextmanager
def deferred_weight_grads(enabled=True):
    """Weight (and bias) gradients of the convs' backward nodes are recorded while this block
    runs a backward pass and computed -- two sources per launch -- when it ends.  Only for
    backward passes whose result is read from .grad (loss.backward(), not autograd.grad),
    and not with gradient hooks on the parameters (they would not fire)."""
    if not enabled or _DEFER[0] is not None:
        yield
        return
    d = _Deferral()
    _DEFER[0] = d
    try:
        yield
    finally:
        _DEFER[0] = None
    _flush_deferred(d)


def _defer_wgrad(weight, X, GY, kind, bias=None) -> bool:
    """Record the pair (X, GY) -- dW += wgrad(X, GY) -- of a leaf `weight` (and, with `bias`,
    that pair's bias gradient sum(GY)) for the end of the active deferred_weight_grads()
    block; False when no block is active or the weight is not a leaf."""
    d = _DEFER[0]
    if d is None or not weight.is_leaf or not weight.requires_grad or not X.is_cuda:
        return False
    e = d.entries.get(id(weight))
    if e is None:
        e = d.entries[id(weight)] = [weight, None, kind, []]
    elif e[2] != kind:
        return False
    if bias is not None:
        if e[1] is not None:
            return False  # a second bias-bearing use: keep the plain path for this one
        e[1] = bias
    e[3].append((X.detach(), GY.detach(), bias is not None))
    return True


def _accum_grad(p, g):
    if p.grad is None:
        p.grad = g
    else:
        p.grad.add_(g)


def _flush_deferred(d):
    with torch.no_grad():
        for w, b, kind, pairs in d.entries.values():
            pairs = sorted(pairs, key=lambda t: not t[2])  # the bias-bearing pair first
            dw, db = _wgrad_pairs(kind, tuple(w.shape), pairs)
            _accum_grad(w, dw)
            if b is not None:
                _accum_grad(b, db)


def _wgrad_one(kind, wshape, X, GY, want_b):
    if kind[0] == "3x3":
        return _wgrad_impl(X, GY, wshape, want_b)
    if kind[0] == "1x1":
        dw, db = _wgrad1x1_raw(GY, X, bool(want_b))
        return dw.view(wshape), db
    return _wgrad_fn(X, GY, wshape, kind[1], bool(want_b))


def _wgrad_separate(kind, wshape, pairs):
    dw = db = None
    for X, GY, hb in pairs:
        w_, b_ = _wgrad_one(kind, wshape, X, GY, hb)
        dw = w_ if dw is None else dw.add_(w_)
        if hb:
            db = b_
    return dw, db


def _two_source_ok(kind, wshape, p1, p2):
    (X1, G1, _), (X2, G2, _) = p1, p2
    if X1.shape[1:] != X2.shape[1:] or G1.shape[1:] != G2.shape[1:]:
        return None
    if X1.dtype != torch.float32 or X2.dtype != torch.float32:
        return None
    N1, C, H, W = X1.shape
    N = N1 + X2.shape[0]
    if kind[0] == "3x3":
        if (_WGRAD and bool(lib.bpk_conv3x3_wino_wgrad_supported(N, C, wshape[0], H, W))
                and (W != 8 or N1 % 2 == 0)):
            return "wino"
        if _IGEMM and _igemm_shape_ok((N, C, H, W), tuple(wshape), (1, 1), (1, 1)):
            return "igemm"
        return None
    if kind[0] == "1x1":
        ok = _IGEMM and _igemm_shape_ok((N, C, H, W), tuple(wshape), (1, 1), (0, 0))
        return "igemm" if ok else None
    cfg = kind[1]
    if _IGEMM and int(cfg[3]) == 1 and _pair(cfg[2]) == (1, 1) and _igemm_shape_ok(
            (N, C, H, W), tuple(wshape), _pair(cfg[0]), _pair(cfg[1])):
        return "igemm"
    return None


def _wgrad_pairs(kind, wshape, pairs):
    if len(pairs) != 2:
        return _wgrad_separate(kind, wshape, pairs)
    how = _two_source_ok(kind, wshape, pairs[0], pairs[1])
    if how is None:
        return _wgrad_separate(kind, wshape, pairs)
    (X1, G1, hb), (X2, G2, _) = pairs
    if how == "wino":
        two = lambda: conv3x3_wgrad2_raw(X1, G1, X2, G2, wshape, hb)  # noqa: E731
    else:
        s, p = {"3x3": ((1, 1), (1, 1)), "1x1": ((1, 1), (0, 0))}.get(kind[0]) or (
            _pair(kind[1][0]), _pair(kind[1][1]))
        two = lambda: conv2d_weight_igemm2_raw(X1, G1, X2, G2, wshape, s, p, hb)  # noqa: E731
    key = ("w2", kind[0], tuple(X1.shape), tuple(X2.shape), tuple(G1.shape), tuple(wshape),
           kind[1] if kind[0] == "gen" else None, bool(hb))
    return _pick_any(key, [two, lambda: _wgrad_separate(kind, wshape, pairs)])


def conv3x3_wgrad2_raw(x, gy, x2, gy2, wshape, bias_grad=False):
    """(dw, db or None): the 3x3 weight gradient summed over two (x, gy) sources in one
    Winograd launch (db: the first source's); == conv3x3_wgrad_raw(x, gy) + (x2, gy2)."""
    x, gy, x2, gy2 = (t.detach().contiguous() for t in (x, gy, x2, gy2))
    N, C, H, W = x.shape
    N2 = x2.shape[0]
    Cout = wshape[0]
    if (tuple(gy.shape) != (N, Cout, H, W) or tuple(x2.shape) != (N2, C, H, W)
            or tuple(gy2.shape) != (N2, Cout, H, W)):
        raise RuntimeError("conv3x3_wgrad2: mismatched sources")
    nbytes = lib.bpk_conv3x3_wino_wgrad_workspace_bytes(N + N2, C, Cout, H, W)
    ws = torch.empty(nbytes // 4, dtype=torch.float32, device=x.device)
    dw = torch.empty((Cout, C, 3, 3), dtype=torch.float32, device=x.device)
    db = torch.empty((Cout,), dtype=torch.float32, device=x.device) if bias_grad else None
    check(lib.bpk_conv3x3_wino_wgrad2_f32(
        x.data_ptr(), gy.data_ptr(), x2.data_ptr(), gy2.data_ptr(), N2, dw.data_ptr(),
        None if db is None else db.data_ptr(), ws.data_ptr(), N, C, Cout, H, W,
        stream_ptr(x.device)), "conv3x3_wgrad2")
    flops.wino3x3("wino_wgrad", N + N2, C, Cout, H, W)
    return dw, db


def conv2d_weight_igemm2_raw(x, gy, x2, gy2, wshape, stride=1, padding=0, bias_grad=False):
    """(dw, db or None) of a general conv summed over two (x, gy) sources in one implicit-GEMM
    launch (db: the first source's)."""
    s, p = _pair(stride), _pair(padding)
    x, gy, x2, gy2 = (t.detach().contiguous() for t in (x, gy, x2, gy2))
    N, C, H, W = x.shape
    N2 = x2.shape[0]
    Co, _, KH, KW = (int(v) for v in wshape)
    Ho, Wo = gy.shape[2], gy.shape[3]
    if tuple(x2.shape[1:]) != (C, H, W) or tuple(gy2.shape) != (N2, Co, Ho, Wo):
        raise RuntimeError("conv2d_igemm_wgrad2: mismatched sources")
    dw = torch.empty((Co, C, KH, KW), dtype=torch.float32, device=x.device)
    db = torch.empty((Co,), dtype=torch.float32, device=x.device) if bias_grad else None
    ws = _igemm_ws(2, N + N2, C, H, W, Co, KH, KW, s, p, Ho, Wo, bias_grad, x.device)
    check(lib.bpk_conv2d_igemm_wgrad2_f32(x.data_ptr(), gy.data_ptr(), x2.data_ptr(),
                                          gy2.data_ptr(), N2, dw.data_ptr(),
                                          None if db is None else db.data_ptr(), ws.data_ptr(),
                                          N, C, H, W, Co, KH, KW, s[0], s[1], p[0], p[1], Ho, Wo,
                                          stream_ptr(x.device)), "conv2d_igemm_wgrad2")
    flops.add("igemm_wgrad", 2.0 * (N + N2) * Co * C * KH * KW * Ho * Wo)
    return dw, db


def _needs_grad(*ts):
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)


def _inference_only(*ts):
    if _needs_grad(*ts):
        raise RuntimeError("conv3x3(pre=...) is inference-only")


def conv3x3_pair(x, x2, weight, bias=None, skip=None, div=1.0, pre=None, stats=False):
    """conv3x3 of the channel concatenation [x, x2] (inference, Winograd kernel) without
    building it; pre / stats as conv3x3."""
    require_hip(x, x2, weight, bias, skip, pre, what="conv3x3_pair")
    _inference_only(x, x2, weight, bias, skip)
    N, C1, H, W = x.shape
    if not (_shape_ok(x, weight[:, :C1]) and C1 % 8 == 0 and bool(lib.bpk_conv3x3_wino_supported(
            N, C1 + x2.shape[1], weight.shape[0], H, W)) and weight.shape[1] == C1 + x2.shape[1]):
        raise RuntimeError(f"conv3x3_pair: unsupported shapes {tuple(x.shape)}, "
                           f"{tuple(x2.shape)} x {tuple(weight.shape)}")
    return conv3x3_fwd_raw(x, weight, bias, skip, div, pre, stats, x2=x2)


def conv3x3(x, weight, bias=None, skip=None, div=1.0, pre=None, stats=False):
    """F.conv2d(x, weight, bias, padding=1) for any fp32 NCHW HIP operands (native kernels
    where the shape qualifies, MIOpen otherwise; every derivative order on 3x3 convs and
    weight gradients), or the residual-block tail
    (skip + conv2d(x, weight, bias)) / div fused into the same launch.  stats=True (inference,
    Winograd path): GroupNorm partial statistics of the output ride along (gn_partials).  With `pre`
    ([N, Cin, 2] from op.norm_act.group_norm_affine) the convolved tensor is
    silu(x * s + t) = act(GroupNorm(x + b)) -- inference only (no autograd)."""
    require_hip(x, weight, bias, skip, pre, what="conv3x3")
    if not _shape_ok(x, weight):
        raise RuntimeError(f"conv3x3: bad operands {tuple(x.shape)} x {tuple(weight.shape)}")
    if pre is not None:
        _inference_only(x, weight, bias, skip)
        if small_supported(x, weight) and weight.shape[0] <= 4:
            y = conv3x3_small_raw(x, weight, bias, pre)
            if skip is not None:
                from .norm_act import residual_rescale
                y = residual_rescale(skip, y, None, div)
            return y
        if not (wino_supported(x, weight) or (not stats and wino_pair_supported(x, weight))):
            raise RuntimeError(f"conv3x3(pre=...): unsupported shape {tuple(x.shape)} x "
                               f"{tuple(weight.shape)}")
        return conv3x3_fwd_raw(x, weight, bias, skip, div, pre, stats)
    if stats and wino_supported(x, weight) and not _needs_grad(x, weight, bias, skip):
        return conv3x3_fwd_raw(x, weight, bias, skip, div, None, stats)
    return _Conv3x3.apply(x, weight, bias, skip, div)


class _GNSiLUConv3x3(torch.autograd.Function):
    """y = (skip + conv3x3(SiLU(GroupNorm(x + bias_nc)), w) + b) / div under autograd, with the
    normalization applied in the Winograd conv's input load (reference layerspp.py:242-274,
    layers.py:626-655: GroupNorm -> act -> Conv), so the normalized activation is never
    stored in the forward.  Backward: the backward-data conv gives d/d(activation); the
    GroupNorm+SiLU backward recomputes the normalization from x and the saved group
    statistics; the weight gradient (only when the engine wants it: DPS differentiates
    w.r.t. the input alone) applies the same (s, t) in its own patch load (or, for shapes the
    Winograd weight gradient does not take, runs on the activation recomputed from them).
    First order only (the score nets are differentiated once).

    `give` / `take` (SkipLink or None): a residual block whose identity skip is the first
    conv's input x hands the skip gradient of its second conv (`give`) to the first conv's
    backward (`take`), which adds it in the GroupNorm backward's pass -- instead of the
    autograd engine accumulating it into x's gradient with a separate full-size add.  The
    engine runs the second conv's backward first (the first conv's output feeds it)."""

    @staticmethod
    def forward(ctx, x, bias_nc, gamma, beta, weight, bias, skip, G, eps, div, stats, give=None,
                take=None, fanout=False):
        from .norm_act import group_norm_affine_stats
        mark_inputs(ctx, x, bias_nc, gamma, beta, weight, bias, skip, G, eps, div, stats, give,
                    take, fanout)
        ctx.give, ctx.take, ctx.fanout = give, take, fanout
        if fanout:
            ctx.set_materialize_grads(False)
        ss, mean, rstd = group_norm_affine_stats(x, G, gamma, beta, eps, bias_nc)
        x = x.detach()
        if gn_partials(x) is None:
            x = x.contiguous()
        y = conv3x3_fwd_raw(x, weight.detach(), bias, skip, div, pre=ss, stats=stats)
        ctx.save_for_backward(x, bias_nc, gamma, beta, weight, mean, rstd, ss)
        ctx.G, ctx.div = G, float(div)
        ctx.has_bias, ctx.has_skip = bias is not None, skip is not None
        # fanout: (y, x) -- the block's input for its 1x1 / conv shortcut, whose gradient then
        # arrives here with gy and joins the GroupNorm backward's pass as its addend
        return (y, x.view_as(x)) if fanout else y

    @staticmethod
    @once_differentiable
    def backward(ctx, gy, dskip=None):
        from .norm_act import ACT_SILU, affine_silu, group_norm_act_backward
        x, bnc, gamma, beta, w, mean, rstd, ss = ctx.saved_tensors
        if gy is None:  # fanout: only the shortcut's gradient came back
            return (dskip,) + (None,) * 13
        gy = gy.contiguous()
        if ctx.div != 1.0:
            gy = gy / ctx.div
        gskip = gy if ctx.has_skip and want_grad(ctx, 6) else None
        if gskip is not None and ctx.give is not None:
            ctx.give.g, gskip = gskip, None  # added by the first conv's GroupNorm backward
        want_w, want_cb = want_grad(ctx, 4), ctx.has_bias and want_grad(ctx, 5)
        gw = gcb = None
        if want_w and wgrad_supported(x, tuple(w.shape)) and not _small_img(x):
            # the activation never stored (small images: materialised below, so the timed
            # Winograd / implicit-GEMM choice of _wgrad_impl still applies)
            r = conv3x3_wgrad_raw(x, gy, tuple(w.shape), bias_grad=want_cb, pre=ss)
            gw, gcb = r if want_cb else (r, None)
        elif want_w:
            gw, gcb = _wgrad_impl(affine_silu(x, ss), gy, tuple(w.shape), want_cb)
        elif want_cb:
            gcb = gy.sum((0, 2, 3))
        dx = d_bnc = dgamma = dbeta = None
        want_x, want_bnc = want_grad(ctx, 0), bnc is not None and want_grad(ctx, 1)
        want_g = gamma is not None and want_grad(ctx, 2)
        want_b = beta is not None and want_grad(ctx, 3)
        addend = None
        if ctx.take is not None:
            addend, ctx.take.g = ctx.take.g, None
            if not want_x:
                addend = None  # x wants no gradient: neither did the skip that sent it
        if dskip is not None:
            addend = dskip if addend is None else addend + dskip
        if want_x or want_bnc or want_g or want_b:
            ga = _fwd_ft_impl(gy, w)
            dx, d_bnc, dgamma, dbeta = group_norm_act_backward(
                ga, x, bnc, gamma, beta, mean, rstd, ctx.G, ACT_SILU, want_bnc, want_g, want_b,
                addend=addend if want_x else None)
        elif dskip is not None:
            dx = dskip
        return dx, d_bnc, dgamma, dbeta, gw, gcb, gskip, None, None, None, None, None, None, None


def gn_silu_conv3x3_ad_supported(x, weight):
    """shapes the autograd GroupNorm+SiLU+conv form takes: the 16-cin Winograd kernel's (with
    the output's GroupNorm partial statistics) or the 8-wide pair form"""
    if x.dim() != 4 or not x.is_cuda or x.dtype != torch.float32 or not _shape_ok(x, weight):
        return False
    if weight.shape[1] > 1024:  # the prologue's GroupNorm table (kPreMaxCin)
        return False
    return wino_supported(x, weight) or (wino_pair_supported(x, weight)
                                         and 2 * weight.shape[1] <= 1024)


class SkipLink:
    """the gradient a residual block's second fused conv hands to its first (see
    _GNSiLUConv3x3): one per block call"""
    __slots__ = ("g",)

    def __init__(self):
        self.g = None


def gn_silu_conv3x3_ad(x, num_groups, gamma, beta, eps, weight, bias=None, skip=None, div=1.0,
                       bias_nc=None, give=None, take=None, fanout=False):
    """(skip + conv3x3(SiLU(GroupNorm(x + bias_nc)), weight) + bias) / div, differentiable
    (first order), the normalization inside the conv's input load; the output carries
    GroupNorm partial statistics for the next GroupNorm when the 16-cin kernel runs.  None
    when the shape does not qualify (gn_silu_conv3x3_ad_supported).  fanout=True: returns
    (y, x), the x for the block's shortcut conv (its gradient is added in this backward)."""
    require_hip(x, weight, bias, skip, bias_nc, what="gn_silu_conv3x3_ad")
    if not gn_silu_conv3x3_ad_supported(x, weight):
        return None
    if skip is not None and tuple(skip.shape) != (x.shape[0], weight.shape[0]) + tuple(x.shape[2:]):
        return None
    stats = bool(wino_supported(x, weight))
    return _GNSiLUConv3x3.apply(x, bias_nc, gamma, beta, weight, bias, skip, num_groups,
                                float(eps), float(div), stats, give, take, bool(fanout))


def up2_supported(x, weight):
    """conv3x3(nearest_x2(x)) on the fused kernel (bpk_conv3x3_wino_up2_f32) for these operands"""
    if not (_WINO_UP2 and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
            and weight.dtype == torch.float32 and tuple(weight.shape[1:]) == (x.shape[1], 3, 3)):
        return False
    N, C, H, W = x.shape
    return bool(lib.bpk_conv3x3_wino_up2_supported(N, C, weight.shape[0], 2 * H, 2 * W))


_WINO_UP2 = True


def _up2_raw(x, weight, bias):
    x = x.detach().contiguous()
    N, C, H, W = x.shape
    Cout = weight.shape[0]
    U = filter_transform(weight, False)
    y = torch.empty((N, Cout, 2 * H, 2 * W), dtype=x.dtype, device=x.device)
    b = None if bias is None else bias.detach().contiguous()
    check(lib.bpk_conv3x3_wino_up2_f32(x.data_ptr(), U.data_ptr(),
                                       None if b is None else b.data_ptr(), y.data_ptr(),
                                       N, C, Cout, 2 * H, 2 * W, stream_ptr(x.device)),
          "conv3x3_wino_up2")
    flops.wino3x3("wino_fwd", N, C, Cout, 2 * H, 2 * W)
    return y


class _Sum2x2(torch.autograd.Function):
    """the sum of each 2 x 2 block (adjoint of the nearest x2 upsample) on the native kernel
    (csrc/channels.hip; aten's strided reduction over the 6-D view took ~470 us per call at
    256^2); its adjoint is the nearest x2 upsample, so higher orders stay recorded ops"""

    @staticmethod
    def forward(ctx, g):
        N, C, H2, W2 = g.shape
        if g.is_cuda and g.dtype == torch.float32:
            g = g.contiguous()
            y = torch.empty((N, C, H2 // 2, W2 // 2), device=g.device, dtype=g.dtype)
            check(lib.bpk_sum2x2_f32(g.data_ptr(), y.data_ptr(), N * C, H2 // 2, W2 // 2,
                                     stream_ptr(g.device)), "sum2x2")
            return y
        return g.reshape(N, C, H2 // 2, 2, W2 // 2, 2).sum((3, 5))

    @staticmethod
    def backward(ctx, gg):
        return F.interpolate(gg, scale_factor=2, mode="nearest")


def _sum2x2(g):
    """adjoint of the nearest x2 upsample: the sum of each 2 x 2 block"""
    if g.shape[2] % 2 or g.shape[3] % 2:
        raise RuntimeError(f"_sum2x2: even spatial sizes expected, got {tuple(g.shape)}")
    return _Sum2x2.apply(g)


class _ConvUp2(torch.autograd.Function):
    """y = conv3x3(nearest_x2(x), w) + b in one launch.  Backward: d/dx = the 2 x 2 block sums
    of the backward-data conv, d/dw = the weight gradient against the upsampled input
    (recomputed), d/db = the sum of gy -- all recorded ops, so higher orders work too."""

    @staticmethod
    def forward(ctx, x, w, b):
        mark_inputs(ctx, x, w, b)
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return _up2_raw(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = gw = gb = None
        if want_grad(ctx, 0):
            gx = _sum2x2(_conv_ft_any(gy, w))
        want_b = ctx.has_bias and want_grad(ctx, 2)
        if want_grad(ctx, 1) or want_b:
            xu = F.interpolate(x, scale_factor=2, mode="nearest")
            if torch.is_grad_enabled():
                gw = _Wgrad3x3.apply(xu, gy, tuple(w.shape)) if want_grad(ctx, 1) else None
                gb = gy.sum((0, 2, 3)) if want_b else None
            else:
                dw, gb = _wgrad_impl(xu, gy, tuple(w.shape), want_b)
                gw = dw if want_grad(ctx, 1) else None
        return gx, gw, gb


def conv3x3_up2(x, weight, bias=None):
    """F.conv2d(F.interpolate(x, scale_factor=2, mode='nearest'), weight, bias, padding=1)
    without materialising the upsampled input (ddpm Upsample, reference layers.py:576-590);
    differentiable.  Raises when up2_supported(x, weight) is False."""
    require_hip(x, weight, bias, what="conv3x3_up2")
    if not up2_supported(x, weight):
        raise RuntimeError(f"conv3x3_up2: unsupported operands {tuple(x.shape)} x {tuple(weight.shape)}")
    if _needs_grad(x, weight, bias):
        return _ConvUp2.apply(x, weight, bias)
    return _up2_raw(x, weight, bias)


def gemm1x1_supported(x, weight, x2=None):
    """The MFMA 1x1-conv GEMM (csrc/gemm_nchw.hip) runs conv1x1([x, x2], weight)."""
    if x.dtype != torch.float32 or weight.dtype != torch.float32 or x.dim() != 4 or not x.is_cuda:
        return False
    N, K1, H, W = x.shape
    K2 = 0 if x2 is None else x2.shape[1]
    if x2 is not None and (x2.shape[0] != N or tuple(x2.shape[2:]) != (H, W)):
        return False
    if weight.shape[1] != K1 + K2 or weight.numel() != weight.shape[0] * (K1 + K2):
        return False
    return bool(lib.bpk_gemm_nchw_supported(N, weight.shape[0], H * W, K1, K2))


def _gemm_nchw(w, ldw, x, K1, x2, K2, b, y, N, M, P):
    """bpk_gemm_nchw_f32, split over K (workspace from the caching allocator) when the launch
    would leave most CUs idle (bpk_gemm_nchw_splitk_bytes > 0)."""
    nws = lib.bpk_gemm_nchw_splitk_bytes(N, M, P, K1, K2)
    ws = torch.empty(nws // 4, dtype=torch.float32, device=x.device) if nws > 0 else None
    check(lib.bpk_gemm_nchw_splitk_f32(w.data_ptr(), ldw, x.data_ptr(), K1,
                                       None if x2 is None else x2.data_ptr(), K2,
                                       None if b is None else b.data_ptr(), y.data_ptr(),
                                       None if ws is None else ws.data_ptr(), N, M, P,
                                       stream_ptr(x.device)), "conv1x1")


def conv1x1(x, weight, bias=None, x2=None):
    """1x1 conv of NCHW x (or of the channel concatenation [x, x2], without building it)
    with weight [Cout, Cin(, 1, 1)] (+ bias): the MFMA GEMM kernel.  Inference only."""
    require_hip(x, weight, bias, x2, what="conv1x1")
    if not gemm1x1_supported(x, weight, x2):
        raise RuntimeError(f"conv1x1: unsupported shape {tuple(x.shape)} x {tuple(weight.shape)}")
    _inference_only(x, weight, bias, x2)
    x = x.contiguous()
    x2 = None if x2 is None else x2.contiguous()
    N, K1, H, W = x.shape
    K2 = 0 if x2 is None else x2.shape[1]
    M = weight.shape[0]
    w = weight.detach().reshape(M, K1 + K2).contiguous()
    b = None if bias is None else bias.detach().contiguous()
    y = torch.empty((N, M, H, W), dtype=torch.float32, device=x.device)
    _gemm_nchw(w, K1 + K2, x, K1, x2, K2, b, y, N, M, H * W)
    flops.add("gemm1x1", 2.0 * N * M * (K1 + K2) * H * W)
    return y


def conv1x1_train_supported(x, weight):
    """The 1x1 GEMM kernels cover conv1x1(x, weight) and all of its derivatives: the forward
    (M = Cout), its adjoint (M = Cin) and the weight gradient (csrc/gemm_nchw.hip)."""
    if (x.dtype != torch.float32 or weight.dtype != torch.float32 or x.dim() != 4
            or not x.is_cuda or weight.dim() not in (2, 4) or tuple(weight.shape[2:]) not in ((), (1, 1))):
        return False
    N, C, H, W = x.shape
    M = weight.shape[0]
    if weight.shape[1] != C:
        return False
    return bool(lib.bpk_gemm_nchw_supported(N, M, H * W, C, 0)
                and lib.bpk_gemm_nchw_supported(N, C, H * W, M, 0)
                and lib.bpk_gemm_nchw_wgrad_supported(N, M, C, H * W))


def _gemm1x1_raw(x, w2d, bias=None):
    """y[n] = w2d @ x[n] (+ bias): the MFMA GEMM, no autograd."""
    x = x.detach().contiguous()
    w = w2d.detach().contiguous()
    N, K, H, W = x.shape
    M = w.shape[0]
    b = None if bias is None else bias.detach().contiguous()
    y = torch.empty((N, M, H, W), dtype=torch.float32, device=x.device)
    _gemm_nchw(w, K, x, K, None, 0, b, y, N, M, H * W)
    flops.add("gemm1x1", 2.0 * N * M * K * H * W)
    return y


def _wgrad1x1_raw(gy, x, bias_grad):
    """(dw [M, K], db [M] or None) = (sum_n gy[n] x[n]^T, gy.sum((0, 2, 3)))."""
    gy = gy.detach().contiguous()
    x = x.detach().contiguous()
    N, K, H, W = x.shape
    M = gy.shape[1]
    nbytes = lib.bpk_gemm_nchw_wgrad_workspace_bytes(N, M, K, H * W)
    ws = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=x.device)
    dw = torch.empty((M, K), dtype=torch.float32, device=x.device)
    db = torch.empty((M,), dtype=torch.float32, device=x.device) if bias_grad else None
    check(lib.bpk_gemm_nchw_wgrad_f32(gy.data_ptr(), x.data_ptr(), dw.data_ptr(),
                                      None if db is None else db.data_ptr(), ws.data_ptr(),
                                      N, M, K, H * W, stream_ptr(x.device)), "conv1x1_wgrad")
    flops.add("gemm1x1_wgrad", 2.0 * N * M * K * H * W)
    return dw, db


def _c1_fn(x, w2d, bias=None):
    if torch.is_grad_enabled():
        return _Conv1x1.apply(x, w2d, bias)
    return _gemm1x1_raw(x, w2d, bias)


def _w1_fn(gy, x, bias_grad):
    if torch.is_grad_enabled():
        return _Wgrad1x1.apply(gy, x, bias_grad)
    return _wgrad1x1_raw(gy, x, bias_grad)


class _Conv1x1(torch.autograd.Function):
    """y = w2d @ x[n] + bias.  Backward: the adjoint is the 1x1 conv with w2d^T, the weight
    and bias gradients one split-K GEMM; all three are differentiable again (PINN residuals
    take second derivatives through the networks)."""

    @staticmethod
    def forward(ctx, x, w2d, bias, wref=None):
        mark_inputs(ctx, x, w2d, bias, wref)
        ctx.save_for_backward(x, w2d)
        # the [Cout, Cin, 1, 1] leaf parameter w2d is a view of (deferred weight gradients)
        ctx.wref = wref
        ctx.bias_leaf = bias if bias is not None and bias.is_leaf else None
        return _gemm1x1_raw(x, w2d, bias)

    @staticmethod
    def backward(ctx, gy):
        x, w2d = ctx.saved_tensors
        gx = None
        if want_grad(ctx, 0):
            if ctx.wref is not None and torch.is_grad_enabled():  # the adjoint, still deferrable
                gx = _Conv1x1.apply(gy, w2d.t(), None, _WRef(ctx.wref.t, not ctx.wref.transposed))
            else:
                gx = _c1_fn(gy, w2d.t())
        gw = gb = None
        want_b = want_grad(ctx, 2)
        # the parameter's gradient from this node: sum gy x^T, or for the adjoint use (w2d is
        # the parameter transposed) sum x gy^T -- the pair (X, GY) = (gy, x)
        pair = (gy, x) if ctx.wref is not None and ctx.wref.transposed else (x, gy)
        if (not torch.is_grad_enabled() and ctx.wref is not None and want_grad(ctx, 1)
                and (not want_b or ctx.bias_leaf is not None)
                and _defer_wgrad(ctx.wref.t, pair[0], pair[1], ("1x1",),
                                 ctx.bias_leaf if want_b else None)):
            pass  # deferred to the end of the backward pass
        elif want_grad(ctx, 1) or want_grad(ctx, 2):
            gw, gb = _w1_fn(gy, x, bool(want_grad(ctx, 2)))
            if not want_grad(ctx, 1):
                gw = None
        return gx, gw, gb, None


class _WRef:
    """A parameter passed to a Function as a plain reference (no autograd edge); transposed:
    the Function's weight is the parameter's transpose (the 1x1 conv's adjoint)."""
    __slots__ = ("t", "transposed")

    def __init__(self, t, transposed=False):
        self.t = t
        self.transposed = transposed


class _Wgrad1x1(torch.autograd.Function):
    """(dw, db) = (sum_n gy[n] x[n]^T, gy.sum((0, 2, 3))); bilinear in (gy, x)."""

    @staticmethod
    def forward(ctx, gy, x, bias_grad):
        mark_inputs(ctx, gy, x, bias_grad)
        ctx.save_for_backward(gy, x)
        return _wgrad1x1_raw(gy, x, bias_grad)

    @staticmethod
    def backward(ctx, ggw, ggb):
        gy, x = ctx.saved_tensors
        g_gy = g_x = None
        if want_grad(ctx, 0):
            if ggw is not None:
                g_gy = _c1_fn(x, ggw, ggb)  # ggw x[n] + ggb
            elif ggb is not None:
                g_gy = ggb.view(1, -1, 1, 1).expand_as(gy)
        if want_grad(ctx, 1) and ggw is not None:
            g_x = _c1_fn(gy, ggw.t())
        return g_gy, g_x, None


def conv1x1_ad(x, weight, bias=None):
    """1x1 conv with autograd on the GEMM kernels (every derivative order); shapes must pass
    conv1x1_train_supported.  weight [Cout, Cin(, 1, 1)]."""
    require_hip(x, weight, bias, what="conv1x1")
    if not conv1x1_train_supported(x, weight):
        raise RuntimeError(f"conv1x1: unsupported shape {tuple(x.shape)} x {tuple(weight.shape)}")
    w2d = weight.reshape(weight.shape[0], weight.shape[1])
    if torch.is_grad_enabled() and weight.is_leaf and weight.dim() == 4:
        return _Conv1x1.apply(x, w2d, bias, _WRef(weight))
    return _c1_fn(x, w2d, bias)


# ---------------------------------------------------------------- general convolutions
# Every other Conv2d / ConvTranspose2d of the networks (stride-2 3x3, the PINN's tiny
# levels and odd channel counts, 2x2 / 4x4 transposed convs, ...) runs through three
# autograd Functions -- conv, its adjoint (conv transpose) and the weight gradient -- whose
# backward passes are written in terms of each other.  Higher derivatives (the PINN
# residual differentiates the networks twice) thus stay plain convolutions, instead of the
# generic convolution double backward, which runs its weight terms as batch/channel-swapped
# convolutions with H x W kernels (0.5-5 ms each on the PINN shapes).  Underneath: the
# implicit-GEMM MFMA kernels (igemm_supported), MIOpen for anything else (groups, dilation).

def _cfg(ctx_like):
    return dict(stride=ctx_like[0], padding=ctx_like[1], dilation=ctx_like[2], groups=ctx_like[3])


def _ig_ok(x, w, cfg):
    return igemm_supported(x, w, cfg[0], cfg[1], cfg[2], cfg[3])


def _conv_fn(x, w, cfg, b=None):
    if torch.is_grad_enabled():
        return _ConvG.apply(x, w, b, cfg)
    return _ConvG.forward(None, x, w, b, cfg)


def _convt_fn(u, w, xshape, cfg):
    if torch.is_grad_enabled():
        return _ConvTG.apply(u, w, xshape, cfg)
    return _ConvTG.forward(None, u, w, xshape, cfg)


def _wgrad_fn(x, gy, wshape, cfg, bias_grad=False):
    """(dw, db or None)"""
    if torch.is_grad_enabled():
        return _WgradG.apply(x, gy, wshape, cfg, bias_grad)
    return _WgradG.forward(None, x, gy, wshape, cfg, bias_grad)


class _ConvG(torch.autograd.Function):
    """y = conv2d(x, w) + b; grads: conv transpose, weight (+ bias) gradient."""

    @staticmethod
    def forward(ctx, x, w, b, cfg):
        mark_inputs(ctx, x, w, b, cfg)
        if ctx is not None:
            ctx.save_for_backward(x, w)
            ctx.cfg = cfg
            ctx.has_b = b is not None
            ctx.bias_leaf = b if b is not None and b.is_leaf else None
        if _ig_ok(x, w, cfg):
            return conv2d_select(x, w, b, cfg[0], cfg[1])
        with torch.no_grad():
            return F.conv2d(x.detach(), w.detach(), None if b is None else b.detach(), **_cfg(cfg))

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = _convt_fn(gy, w, tuple(x.shape), ctx.cfg) if want_grad(ctx, 0) else None
        gw = gb = None
        want_b = ctx.has_b and want_grad(ctx, 2)
        if (not torch.is_grad_enabled() and want_grad(ctx, 1)
                and (not want_b or ctx.bias_leaf is not None)
                and _defer_wgrad(w, x, gy, ("gen", ctx.cfg), ctx.bias_leaf if want_b else None)):
            pass  # deferred to the end of the backward pass
        elif want_grad(ctx, 1) or want_b:
            gw, gb = _wgrad_fn(x, gy, tuple(w.shape), ctx.cfg, bool(want_b))
            if not want_grad(ctx, 1):
                gw = None
        return gx, gw, gb, None


class _ConvTG(torch.autograd.Function):
    """z = conv2d's adjoint w.r.t. its input: z = A_w^T u (shape xshape)."""

    @staticmethod
    def forward(ctx, u, w, xshape, cfg):
        mark_inputs(ctx, u, w, xshape, cfg)
        if ctx is not None:
            ctx.save_for_backward(u, w)
            ctx.cfg = cfg
        if (_IGEMM and u.is_cuda and u.dtype == torch.float32 and w.dtype == torch.float32
                and int(cfg[3]) == 1 and _pair(cfg[2]) == (1, 1)
                and _igemm_shape_ok(tuple(int(v) for v in xshape), tuple(w.shape),
                                    _pair(cfg[0]), _pair(cfg[1]))):
            return conv2d_input_select(xshape, w, u, cfg[0], cfg[1])
        with torch.no_grad():
            return torch.nn.grad.conv2d_input(xshape, w.detach(), u.detach(), **_cfg(cfg))

    @staticmethod
    def backward(ctx, gz):
        u, w = ctx.saved_tensors
        gu = _conv_fn(gz, w, ctx.cfg) if want_grad(ctx, 0) else None
        gw = None
        if want_grad(ctx, 1) and (torch.is_grad_enabled()
                                  or not _defer_wgrad(w, gz, u, ("gen", ctx.cfg))):
            gw = _wgrad_fn(gz, u, tuple(w.shape), ctx.cfg)[0]
        return gu, gw, None, None


class _WgradG(torch.autograd.Function):
    """(dw, db) = d<conv2d(x, w) + b, gy>/d(w, b); bilinear in (x, gy)."""

    @staticmethod
    def forward(ctx, x, gy, wshape, cfg, bias_grad):
        mark_inputs(ctx, x, gy, wshape, cfg, bias_grad)
        if ctx is not None:
            ctx.save_for_backward(x, gy)
            ctx.cfg = cfg
        if _ig_ok(x, tuple(wshape), cfg):
            return conv2d_weight_select(x, wshape, gy, cfg[0], cfg[1], bias_grad)
        with torch.no_grad():
            dw = torch.nn.grad.conv2d_weight(x.detach(), wshape, gy.detach(), **_cfg(cfg))
            return dw, (gy.detach().sum((0, 2, 3)) if bias_grad else None)

    @staticmethod
    def backward(ctx, ggw, ggb):
        x, gy = ctx.saved_tensors
        gx = ggy = None
        if want_grad(ctx, 0) and ggw is not None:
            gx = _convt_fn(gy, ggw, tuple(x.shape), ctx.cfg)
        if want_grad(ctx, 1):
            if ggw is not None:
                ggy = _conv_fn(x, ggw, ctx.cfg, ggb)
            elif ggb is not None:
                ggy = ggb.view(1, -1, 1, 1).expand_as(gy)
        return gx, ggy, None, None, None


def conv2d_general(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1):
    """F.conv2d with every derivative order expressed as convolutions / conv transposes /
    weight gradients (see above); bias fused into the forward and weight-gradient kernels."""
    cfg = (_pair(stride), _pair(padding), _pair(dilation), int(groups))
    return _conv_fn(x, weight, cfg, bias)


def _dense_groups(w, groups):
    """ConvTranspose2d weight [Cin, Cout / g, k, k] -> the block-diagonal dense weight
    [Cin, Cout, k, k] (differentiable; the FlowNet flow upsample has g = 2 channels)."""
    if groups == 1:
        return w
    ci, cog, kh, kw = w.shape
    wv = w.reshape(groups, ci // groups, cog, kh, kw)
    eye = torch.eye(groups, dtype=w.dtype, device=w.device)
    return torch.einsum("aijkl,ab->aibjkl", wv, eye).reshape(ci, groups * cog, kh, kw)


def conv_transpose2d_general(u, weight, bias=None, stride=1, padding=0, output_padding=0,
                             groups=1, dilation=1):
    """F.conv_transpose2d(u, weight, bias, stride, padding, output_padding, groups, dilation)
    as the adjoint of conv2d(., weight) (the dgrad kernel), every derivative order on the
    same three Functions; groups through a block-diagonal dense weight."""
    s, p, op, d = _pair(stride), _pair(padding), _pair(output_padding), _pair(dilation)
    w = _dense_groups(weight, int(groups))
    N, _, Hu, Wu = u.shape
    Ho = (Hu - 1) * s[0] - 2 * p[0] + d[0] * (w.shape[2] - 1) + op[0] + 1
    Wo = (Wu - 1) * s[1] - 2 * p[1] + d[1] * (w.shape[3] - 1) + op[1] + 1
    y = _convt_fn(u, w, (N, w.shape[1], Ho, Wo), (s, p, d, 1))
    return y if bias is None else y + bias.view(1, -1, 1, 1)
