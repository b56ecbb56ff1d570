"""Do independent branches of a captured hipGraph run concurrently on this stack?  Two chains of
N tiny dependent kernels, captured (a) both on one stream, (b) on two forked streams joined at the
end; replay times of each (and of one chain alone)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
from op import _hipenv  # noqa: E402,F401
import torch  # noqa: E402

dev = torch.device("cuda:0")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 500
a = torch.zeros(4096, device=dev)
b = torch.zeros(4096, device=dev)


def chain(t, n):
    for _ in range(n):
        t.add_(1.0)


def capture(fn):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def one():
    chain(a, N)


def serial():
    chain(a, N)
    chain(b, N)


side = torch.cuda.Stream(dev)


def forked():
    cur = torch.cuda.current_stream(dev)
    side.wait_stream(cur)
    chain(a, N)
    with torch.cuda.stream(side):
        chain(b, N)
    cur.wait_stream(side)


def timed(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


res = {}
for name, fn in (("one_chain", one), ("two_chains_serial", serial), ("two_chains_forked", forked)):
    g = capture(fn)
    res[name] = round(timed(g), 3)
print({"kernels_per_chain": N, "replay_ms": res,
       "us_per_kernel_one_chain": round(res["one_chain"] / N * 1e3, 2)})
