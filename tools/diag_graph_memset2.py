"""hipMemsetAsync nodes and aten's global (multi-block) reduction under hipGraph replay,
with and without a side-stream warm-up before the capture."""
import ctypes

import torch

dev = torch.device("cuda:0")
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]


def memset_case(side, nbytes):
    buf = torch.empty(nbytes // 4, device=dev)
    out = torch.empty_like(buf)

    def body():
        hip.hipMemsetAsync(buf.data_ptr(), 0, nbytes, torch.cuda.current_stream().cuda_stream)
        buf.add_(1.0)
        out.copy_(buf)
    if side:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body()
        torch.cuda.current_stream().wait_stream(s)
    else:
        body()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    vals = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        vals.append(float(out.max()))
    print(f"memset side={side} {nbytes} B: out max per replay {vals} (expect 1.0)", flush=True)


def reduce_case(side, shape):
    a = torch.randn(*shape, device=dev)
    ref = a.sum((0, 2, 3))
    res = {}

    def body():
        res["y"] = a.sum((0, 2, 3))
    if side:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body()
        torch.cuda.current_stream().wait_stream(s)
    else:
        body()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    d = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        d.append("%.2e" % float((res["y"] - ref).abs().max()))
    print(f"sum((0,2,3)) side={side} {shape}: |graph - eager| per replay {d}", flush=True)


for side in (False, True):
    for nb in (16, 1536, 1 << 20):
        memset_case(side, nb)
    for shape in ((64, 6, 64, 64), (64, 32, 64, 64), (4, 6, 16, 16)):
        reduce_case(side, shape)
