"""Topology of a captured hipGraph (torch.cuda.CUDAGraph(keep_graph=True)): node count, root
nodes, edges, node types, and whether it is the single chain a one-stream capture should give."""
import collections
import ctypes

_hip = ctypes.CDLL("libamdhip64.so")
_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty",
          6: "wait_event", 7: "event_record", 8: "ext_sem_signal", 9: "ext_sem_wait",
          10: "mem_alloc", 11: "mem_free", 12: "memcpy1d", 13: "memcpy_from_symbol",
          14: "memcpy_to_symbol"}


def topology(raw_graph):
    g = ctypes.c_void_p(raw_graph)
    n = ctypes.c_size_t(0)
    assert _hip.hipGraphGetNodes(g, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert _hip.hipGraphGetNodes(g, nodes, ctypes.byref(n)) == 0
    r = ctypes.c_size_t(0)
    assert _hip.hipGraphGetRootNodes(g, None, ctypes.byref(r)) == 0
    e = ctypes.c_size_t(0)
    assert _hip.hipGraphGetEdges(g, None, None, ctypes.byref(e)) == 0
    frm = (ctypes.c_void_p * max(e.value, 1))()
    to = (ctypes.c_void_p * max(e.value, 1))()
    if e.value:
        assert _hip.hipGraphGetEdges(g, frm, to, ctypes.byref(e)) == 0
    outdeg = collections.Counter(frm[i] for i in range(e.value))
    indeg = collections.Counter(to[i] for i in range(e.value))
    types = collections.Counter()
    for i in range(n.value):
        t = ctypes.c_int(0)
        _hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t))
        types[_TYPES.get(t.value, t.value)] += 1
    fan_out = sum(1 for v in outdeg.values() if v > 1)
    fan_in = sum(1 for v in indeg.values() if v > 1)
    return {"nodes": n.value, "roots": r.value, "edges": e.value, "fan_out_nodes": fan_out,
            "fan_in_nodes": fan_in, "chain": r.value == 1 and e.value == n.value - 1 and not fan_out,
            "types": dict(types)}


class _Pos(ctypes.Structure):
    _fields_ = [("x", ctypes.c_size_t), ("y", ctypes.c_size_t), ("z", ctypes.c_size_t)]


class _Pitched(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("pitch", ctypes.c_size_t), ("xsize", ctypes.c_size_t),
                ("ysize", ctypes.c_size_t)]


class _Extent(ctypes.Structure):
    _fields_ = [("width", ctypes.c_size_t), ("height", ctypes.c_size_t),
                ("depth", ctypes.c_size_t)]


class _Memcpy3D(ctypes.Structure):
    _fields_ = [("srcArray", ctypes.c_void_p), ("srcPos", _Pos), ("srcPtr", _Pitched),
                ("dstArray", ctypes.c_void_p), ("dstPos", _Pos), ("dstPtr", _Pitched),
                ("extent", _Extent), ("kind", ctypes.c_int)]


class _Memset(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_void_p), ("elementSize", ctypes.c_uint), ("height", ctypes.c_size_t),
                ("pitch", ctypes.c_size_t), ("value", ctypes.c_uint), ("width", ctypes.c_size_t)]


def copy_nodes(raw_graph):
    """[(order, 'memcpy', src, dst, bytes, kind) / (order, 'memset', dst, bytes, value)] in
    chain order."""
    g = ctypes.c_void_p(raw_graph)
    n = ctypes.c_size_t(0)
    _hip.hipGraphGetNodes(g, None, ctypes.byref(n))
    nodes = (ctypes.c_void_p * n.value)()
    _hip.hipGraphGetNodes(g, nodes, ctypes.byref(n))
    e = ctypes.c_size_t(0)
    _hip.hipGraphGetEdges(g, None, None, ctypes.byref(e))
    frm = (ctypes.c_void_p * max(e.value, 1))()
    to = (ctypes.c_void_p * max(e.value, 1))()
    if e.value:
        _hip.hipGraphGetEdges(g, frm, to, ctypes.byref(e))
    nxt = {frm[i]: to[i] for i in range(e.value)}
    r = ctypes.c_size_t(1)
    root = (ctypes.c_void_p * 1)()
    _hip.hipGraphGetRootNodes(g, root, ctypes.byref(r))
    order, cur = [], root[0]
    while cur is not None:
        order.append(cur)
        cur = nxt.get(cur)
    out = []
    for i, nd in enumerate(order):
        t = ctypes.c_int(0)
        _hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
        if t.value == 1:
            p = _Memcpy3D()
            _hip.hipGraphMemcpyNodeGetParams(ctypes.c_void_p(nd), ctypes.byref(p))
            nbytes = p.extent.width * max(p.extent.height, 1) * max(p.extent.depth, 1)
            out.append((i, "memcpy", p.srcPtr.ptr or 0, p.dstPtr.ptr or 0, nbytes, p.kind))
        elif t.value == 2:
            p = _Memset()
            _hip.hipGraphMemsetNodeGetParams(ctypes.c_void_p(nd), ctypes.byref(p))
            out.append((i, "memset", p.dst or 0, p.width * max(p.height, 1) * p.elementSize,
                        p.value))
    return out, len(order)


def classify(ptr, segments):
    for s in segments:
        if s["address"] <= ptr < s["address"] + s["total_size"]:
            return f"pool{tuple(s.get('segment_pool_id', ()))}"
    return "not-torch"
