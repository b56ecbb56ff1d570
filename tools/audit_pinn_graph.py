"""Audit of the captured PINN train step (losses._PinnGraphStep) -- VERDICT r04 item 1.

    python tools/audit_pinn_graph.py audit [B]        -> gpurun_out/pinn_graph_audit.json
    python tools/audit_pinn_graph.py iso MODE [B]     -> fixed-parameter replays with MODE's
                                                         eager work between them

`audit` captures the step with three probes on:
  * every aten op executed during the capture (a TorchDispatchMode, which the autograd engine
    carries into its worker thread) and every libbpk C-ABI call: the device pointers each one
    passes, and how many graph nodes of each type (kernel / memset / memcpy / ...) the call
    added to the capture (hipStreamGetCaptureInfo_v2 + hipGraphGetNodes before and after);
  * after the capture, every logged pointer is located in torch.cuda.memory_snapshot(): in the
    graph's private pool, in a live eager block, in a FREE eager block (a bug), or outside the
    caching allocator (a bug unless explained);
  * CPU-sourced copies recorded in the capture (an aten op mixing host and device tensors).

`iso MODE` replays the captured step with the parameters, inputs and noise fixed (every replay
must give bit-identical losses) and runs MODE between replays:
  none | memset0 (hipMemsetAsync of eager scratch, value 0) | memsetx (value 0x5a) |
  redlarge (sums of 300k-element tensors kept on the device: global reductions) |
  redsmall (sums of 1000-element tensors) | d2h (float() of single elements) |
  redlarge_item (r04's failing case: large sums read back with float()) |
  fillflood (2000 small-argument fill kernels) | ncflood (200 non-contiguous adds: large
  kernel-argument blocks, no reduction).
`pc MODE` runs the PC sampler's step graph (bench config, B=8) for 24 steps twice -- with and
without MODE's eager work between the steps -- and compares the trajectories bit for bit
(the noise is counter-based, so they must agree).
"""
import ctypes
import json
import os
import sys
from collections import Counter, defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402
from torch.utils._pytree import tree_flatten  # noqa: E402

import bench  # noqa: E402
import losses  # noqa: E402
from configs.pinn import pinn_pde  # noqa: E402
from inverse.operators import get_operator  # noqa: E402
from op import _lib  # noqa: E402
from pinn_kalman.pinn import PINN  # noqa: E402

OUT = os.path.join(REPO, "gpurun_out")
NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty",
              6: "wait_event", 7: "event_record", 8: "ext_sem_signal", 9: "ext_sem_wait",
              10: "mem_alloc", 11: "mem_free", 12: "memcpy_from_symbol", 13: "memcpy_to_symbol"}


def _hip():
    for line in open("/proc/self/maps"):
        if "libamdhip64.so" in line:
            return ctypes.CDLL(line.split()[-1])
    raise RuntimeError("libamdhip64 not loaded")


class Capture:
    """Graph-node accounting of the capture running on `stream`."""

    def __init__(self, hip):
        self.hip = hip
        hip.hipStreamGetCaptureInfo_v2.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                                   ctypes.POINTER(ctypes.c_ulonglong),
                                                   ctypes.POINTER(ctypes.c_void_p),
                                                   ctypes.POINTER(ctypes.c_void_p),
                                                   ctypes.POINTER(ctypes.c_size_t)]
        hip.hipGraphGetNodes.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.POINTER(ctypes.c_size_t)]
        hip.hipGraphNodeGetType.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]

    def graph_of(self, stream):
        st, cid, g = ctypes.c_int(0), ctypes.c_ulonglong(0), ctypes.c_void_p(0)
        deps, nd = ctypes.c_void_p(0), ctypes.c_size_t(0)
        if self.hip.hipStreamGetCaptureInfo_v2(ctypes.c_void_p(stream), ctypes.byref(st),
                                              ctypes.byref(cid), ctypes.byref(g),
                                              ctypes.byref(deps), ctypes.byref(nd)) != 0:
            return None
        return g.value if st.value == 1 else None

    def count(self, graph):
        n = ctypes.c_size_t(0)
        self.hip.hipGraphGetNodes(ctypes.c_void_p(graph), None, ctypes.byref(n))
        return n.value

    def nodes(self, graph, start=0):
        """the graph's nodes[start:] (hipGraphGetNodes lists them in creation order)"""
        n = ctypes.c_size_t(self.count(graph))
        arr = (ctypes.c_void_p * max(n.value, 1))()
        self.hip.hipGraphGetNodes(ctypes.c_void_p(graph), arr, ctypes.byref(n))
        return list(arr[start:n.value])

    def types(self, nodes):
        out = Counter()
        for nd in nodes:
            t = ctypes.c_int(-1)
            self.hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
            out[NODE_TYPES.get(t.value, str(t.value))] += 1
        return out


class Recorder:
    def __init__(self, cap):
        self.cap = cap
        self.on = False
        self.events = []  # (kind, name, [ptrs], node-type counts, host_sourced)

    def around(self, kind, name, ptrs, fn, host=False):
        if not (self.on and torch.cuda.is_current_stream_capturing()):
            return fn()
        stream = torch.cuda.current_stream().cuda_stream
        g = self.cap.graph_of(stream)
        n0 = self.cap.count(g) if g else 0
        out = fn()
        new = self.cap.nodes(g, n0) if g and self.cap.count(g) > n0 else []
        extra = out if kind == "aten" else None
        optrs = []
        if extra is not None:
            for t in tree_flatten(extra)[0]:
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    optrs.append((t.untyped_storage().data_ptr(), t.untyped_storage().nbytes()))
        self.events.append(dict(kind=kind, name=name, ptrs=ptrs, out=optrs,
                                nodes=dict(self.cap.types(new)), host_sourced=host))
        return out


def _tensor_ptrs(args, kwargs):
    ptrs, host = [], False
    flat = tree_flatten((args, kwargs))[0]
    has_dev = any(isinstance(t, torch.Tensor) and t.is_cuda for t in flat)
    for t in flat:
        if isinstance(t, torch.Tensor):
            if t.is_cuda:
                ptrs.append((t.untyped_storage().data_ptr(), t.untyped_storage().nbytes()))
            elif has_dev and t.numel() > 0 and not (t.dim() == 0):
                host = True
    return ptrs, host


class AtenProbe(TorchDispatchMode):
    def __init__(self, rec):
        super().__init__()
        self.rec = rec

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        ptrs, host = _tensor_ptrs(args, kwargs)
        return self.rec.around("aten", str(func), ptrs, lambda: func(*args, **kwargs), host)


def probe_cabi(rec):
    orig = _lib._Lib.__getattr__

    def ga(self, name):
        fn = orig(self, name)
        if not name.startswith("bpk_") or self._protos is None or name not in self._protos:
            return fn
        argtypes = self._protos[name][1]

        def wrapped(*a):
            ptrs = [(int(v), 0) for v, ty in zip(a[:-1], argtypes[:-1])
                    if ty is ctypes.c_void_p and v]
            return rec.around("cabi", name, ptrs, lambda: fn(*a))
        return wrapped
    _lib._Lib.__getattr__ = ga


def locate(snapshot, graph_pools):
    segs = []
    for s in snapshot:
        blocks, addr = [], s["address"]
        for b in s["blocks"]:
            a = b.get("address", addr)
            blocks.append((a, a + b["size"], b["state"], b.get("frames", [])))
            addr = a + b["size"]
        segs.append((s["address"], s["address"] + s["total_size"],
                     tuple(s.get("segment_pool_id", (0, 0))), blocks))

    def where(p):
        for lo, hi, pool, blocks in segs:
            if lo <= p < hi:
                if pool in graph_pools:
                    return "graph_pool", None
                for blo, bhi, state, frames in blocks:
                    if blo <= p < bhi:
                        fr = [f"{f.get('filename', '?').split('/')[-1]}:{f.get('line', '?')}"
                              f" {f.get('name', '')}" for f in frames[:6]]
                        if state == "active_allocated":
                            return "eager_live", (blo, fr)
                        return f"eager_{state}", (blo, fr)
                return "eager_unmapped_block", None
        return "outside_allocator", None
    return where


def build(B):
    dev = torch.device("cuda:0")
    c = pinn_pde.get_config()
    c.device = dev
    c.training.batch_size = B
    torch.manual_seed(0)
    model = PINN(c)
    model.train()
    fn = losses.get_pinn_step_fn(c, train=True, optimize_fn=losses.optimization_manager(c),
                                 graph=True)
    operator = get_operator(c)
    operator.next()
    batch = bench.pinn_batch(c, B, dev, seed=0)
    return dev, c, model, fn, operator, batch


def owners(model, fn):
    """storage pointer -> name of the live eager tensors the graph is expected to read."""
    out = {}

    def add(name, t):
        if isinstance(t, torch.Tensor) and t.is_cuda:
            out[t.untyped_storage().data_ptr()] = name
    for n, p in model.named_parameters():
        add("param " + n, p)
        for attr in ("_bpk_wino_u", "_bpk_wino_u_ft"):
            if getattr(p, attr, None) is not None:
                add(f"wino U cache {n}", getattr(p, attr)[1])
    for n, b in model.named_buffers():
        add("buffer " + n, b)
    for i, t in enumerate(fn.static):
        add(f"static batch[{i}]", t)
    add("static mask", fn.mask)
    for i, t in enumerate(fn.noise):
        add(f"static noise[{i}]", t)
    add("obuf", fn.obuf)
    for p in fn.params:
        if p.grad is not None:
            add("eager gbuf", p.grad)
    from models import flownet
    for k, g in flownet._BASE_GRIDS.items():
        add(f"flownet base grid {k}", g)
    return out


def audit(B):
    hip = _hip()
    cap = Capture(hip)
    rec = Recorder(cap)
    probe_cabi(rec)
    torch.cuda.memory._record_memory_history(max_entries=200000)
    dev, c, model, fn, operator, batch = build(B)
    graphs = []
    orig_graph = torch.cuda.graph

    class probed:
        def __init__(self, g, *a, **k):
            self.g, self.cm, self.mode = g, orig_graph(g, *a, **k), AtenProbe(rec)
            graphs.append(g)

        def __enter__(self):
            r = self.cm.__enter__()
            rec.on = True
            self.mode.__enter__()
            return r

        def __exit__(self, *e):
            self.mode.__exit__(*e)
            rec.on = False
            return self.cm.__exit__(*e)
    torch.cuda.graph = probed
    try:
        fn._capture(model, operator, batch)
    finally:
        torch.cuda.graph = orig_graph
    torch.cuda.synchronize()
    totals = []
    for g in graphs:
        try:
            totals.append(dict(cap.types(cap.nodes(g.raw_cuda_graph()))))
        except Exception as e:  # noqa: BLE001
            totals.append({"error": repr(e)})
    pools = {tuple(g.pool()) for g in graphs}
    where = locate(torch.cuda.memory_snapshot(), pools)
    own = owners(model, fn)
    cls = Counter()
    flagged, live = [], defaultdict(int)
    node_by_op = defaultdict(Counter)
    host_ops = Counter()
    for ev in rec.events:
        for k, v in ev["nodes"].items():
            node_by_op[ev["name"]][k] += v
        if ev["host_sourced"]:
            host_ops[ev["name"]] += 1
        for p, _n in ev["ptrs"]:
            w, info = where(p)
            cls[w] += 1
            if w == "eager_live":
                blo = info[0]
                live[own.get(blo, own.get(p, "UNKNOWN live block @%x: %s" % (blo, info[1])))] += 1
            elif w != "graph_pool":
                flagged.append(dict(op=ev["name"], ptr=hex(p), where=w,
                                    frames=None if info is None else info[1]))
    memset_ops = {k: dict(v) for k, v in node_by_op.items() if v.get("memset") or v.get("memcpy")}
    rep = dict(batch=B, graphs=totals, pointer_classes=dict(cls),
               flagged=flagged[:200], n_flagged=len(flagged),
               live_eager_reads=dict(sorted(live.items())),
               unknown_live=[k for k in live if k.startswith("UNKNOWN")],
               host_sourced_ops=dict(host_ops),
               ops_adding_memset_or_memcpy_nodes=memset_ops,
               n_events=len(rec.events))
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "pinn_graph_audit.json"), "w") as f:
        json.dump(rep, f, indent=1)
    print(json.dumps({k: rep[k] for k in ("graphs", "pointer_classes", "n_flagged",
                                          "unknown_live", "host_sourced_ops",
                                          "ops_adding_memset_or_memcpy_nodes")}, indent=1))


def iso(mode, B):
    hip = _hip()
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    dev, c, model, fn, operator, batch = build(B)
    fn._capture(model, operator, batch)
    with torch.no_grad():
        for d, b in zip(fn.static, batch):
            d.copy_(b)
        fn.mask.copy_(operator.mask.to(dev))
        for z in fn.noise:
            z.normal_()
    scratch = torch.empty(1 << 22, device=dev)
    keep, ref, bad, ms = [], None, [], []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(20):
        e0.record()
        fn.graph.replay()
        e1.record()
        vals = [float(t) for t in fn.out]
        ms.append(e0.elapsed_time(e1))
        ref = vals if ref is None else ref
        if vals != ref:
            bad.append(i)
        print(mode, i, vals, flush=True)
        eager_work(mode, hip, scratch, keep, dev)
        torch.cuda.synchronize()
        if len(keep) > 400:
            del keep[:200]
    ms = sorted(ms)
    res = dict(mode=mode, batch=B, stable=not bad, first_bad=bad[0] if bad else None,
               replay_ms_median=round(ms[len(ms) // 2], 3),
               env={k: os.environ.get(k) for k in ENV_KNOBS if os.environ.get(k) is not None})
    print("RESULT", json.dumps(res), flush=True)


ENV_KNOBS = ("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "HIP_FORCE_DEV_KERNARG", "HSA_KERNARG_POOL_SIZE",
             "DEBUG_HIP_KERNARG_COPY_OPT")


def eager_work(mode, hip, scratch, keep, dev):
    if mode == "fillflood":
        for k in range(2000):
            scratch[:1024].fill_(float(k))
        return
    if mode == "ncflood":
        a = scratch[:1 << 20].view(1024, 1024)
        for _ in range(200):
            b = a.t() + a  # noqa: F841
        return
    for k in range(1, 40):
        n = (k * 7919) % 300000 + 1
        if mode == "memset0" or mode == "memsetx":
            hip.hipMemsetAsync(ctypes.c_void_p(scratch.data_ptr()), 0 if mode == "memset0" else 0x5a,
                               ctypes.c_size_t(4 * min(n, scratch.numel())),
                               ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        elif mode == "redlarge":
            keep.append(torch.randn(n, device=dev).double().abs().sum())
        elif mode == "redsmall":
            keep.append(torch.randn(1000, device=dev).sum())
        elif mode == "d2h":
            float(scratch[k])
        elif mode == "redlarge_item":
            float(torch.randn(n, device=dev).double().abs().sum())


def pc(mode, B=8, steps=24):
    hip = _hip()
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    import sampling
    import sde_lib
    dev = torch.device("cuda:0")
    c, model = bench.build_model(dev)
    model.eval()
    sde = sde_lib.VPSDE(c.model.beta_min, c.model.beta_max, c.model.num_scales)
    scratch = torch.empty(1 << 22, device=dev)
    keep, outs = [], []
    prior = torch.randn(B, 1, 128, 128, generator=torch.Generator().manual_seed(5))
    for work in (False, True):
        eng = sampling.PCEngine(sde, (B, 1, 128, 128), sampling.EulerMaruyamaPredictor,
                                sampling.LangevinCorrector, c.sampling.snr, 1, continuous=True,
                                device=dev, seed=1234)
        eng.reset(model, x_init=prior)  # the same prior in both runs (round 5's first pc
        for _ in range(steps):            # run drew two different priors: not a graph effect)
            eng.advance(1)
            if work:
                eager_work(mode, hip, scratch, keep, dev)
        torch.cuda.synchronize()
        outs.append(eng._xm.clone())
        del eng
    same = bool(torch.equal(outs[0], outs[1]))
    print("RESULT", json.dumps(dict(pc_mode=mode, batch=B, steps=steps, identical=same,
                                    max_abs_diff=float((outs[0] - outs[1]).abs().max()),
                                    env={k: os.environ.get(k) for k in ENV_KNOBS
                                         if os.environ.get(k) is not None})), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "audit":
        audit(int(sys.argv[2]) if len(sys.argv) > 2 else 64)
    elif sys.argv[1] == "pc":
        pc(sys.argv[2])
    else:
        iso(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 64)
